"""auto_parallel.static.engine.Engine (reference: python/paddle/distributed/auto_parallel/static/
engine.py:68): the high-level fit / evaluate / predict / save / load API over a DistModel.

The reference's Engine plans a distributed static program (completion, partitioner, reshard) from
the model and its strategy.  Here the step is dist.to_static's DistModel: data-parallel, gradient
merge, AMP, sharding stage 1/2/3 and pipeline stages (parameters placed on per-stage process
meshes) are recorded into a static Program and replayed by the Executor on each rank, with the
gradient reduce-scatter / all-reduce and the stage-to-stage activation exchange as the program's
collectives; what the program form does not cover (tensor-parallel Shard placements, recompute)
runs the same step eagerly on the SPMD-propagated dist tensors.
"""
import torch.distributed as dist

from ..api import DistModel, Strategy


class Engine:
    """Auto-parallel high-level API (reference: distributed/auto_parallel/static/engine.py:68,
    ``from paddle.distributed.fleet import auto; auto.Engine``): ``fit`` / ``evaluate`` /
    ``predict`` / ``save`` / ``load`` over a DistModel (strategy: sharding, gradient merge,
    pipeline micro-batching, AMP, recompute).  The reference compiles a distributed static
    program; here the step runs eagerly on the SPMD-propagated dist tensors, so the placements
    given with shard_tensor / shard_layer drive the collectives.  Data: each rank reads its
    data-parallel share of every batch (DistributedBatchSampler over the world) unless the
    dataset is already split."""

    def __init__(self, model=None, loss=None, optimizer=None, metrics=None, cluster=None, strategy=None):
        self._model = model
        self._loss = loss
        self._optimizer = optimizer
        self._metrics = [] if metrics is None else (list(metrics) if isinstance(metrics, (list, tuple)) else [metrics])
        self._strategy = strategy if strategy is not None else Strategy()
        self._dm = None
        self._mode = 'train'
        self.history = None

    # -- plumbing
    def _dist_model(self):
        if self._dm is None:
            self._dm = DistModel(self._model, None, self._loss, self._optimizer, self._strategy)
        return self._dm

    def _loader(self, data, batch_size, collate_fn, shuffle=False):
        from ....io import DataLoader, Dataset, DistributedBatchSampler
        if data is None:
            return None
        if not isinstance(data, Dataset):
            return data  # an iterable of ready batches
        if batch_size is None:
            return data
        if dist.is_initialized() and dist.get_world_size() > 1:
            bs = DistributedBatchSampler(data, batch_size=batch_size, shuffle=shuffle, drop_last=True)
            return DataLoader(data, batch_sampler=bs, collate_fn=collate_fn)
        return DataLoader(data, batch_size=batch_size, shuffle=shuffle, collate_fn=collate_fn, drop_last=False)

    @staticmethod
    def _split(batch, split):
        items = list(batch) if isinstance(batch, (list, tuple)) else [batch]
        k = split if split is not None else (len(items) - 1 if len(items) > 1 else len(items))
        return items[:k], items[k:]

    def _update_metrics(self, out, labels):
        res = {}
        for m in self._metrics:
            r = m.compute(out, *labels) if hasattr(m, 'compute') else out
            m.update(*(r if isinstance(r, (list, tuple)) else [r]))
            acc = m.accumulate()
            names = m.name() if callable(getattr(m, 'name', None)) else [type(m).__name__]
            names = names if isinstance(names, (list, tuple)) else [names]
            vals = acc if isinstance(acc, (list, tuple)) else [acc]
            res.update(dict(zip(names, vals)))
        return res

    # -- public API
    def prepare(self, inputs_spec=None, labels_spec=None, inputs=None, labels=None, main_program=None,
                startup_program=None, mode='train', init_parameters=True):
        self._mode = mode
        self._dist_model()

    def to_mode(self, mode):
        assert mode in ('train', 'eval', 'predict'), mode
        self._mode = mode

    def fit(self, train_data, train_sample_split=None, batch_size=1, epochs=1, steps_per_epoch=None, log_freq=10,
            save_dir=None, save_freq=1, valid_data=None, valid_sample_split=None, valid_freq=1, valid_steps=None,
            collate_fn=None, callbacks=None, verbose=2, nvprof_range=(-1, -1)):
        dm = self._dist_model()
        self._mode = 'train'
        loader = self._loader(train_data, batch_size, collate_fn, shuffle=False)
        history = {'loss': []}
        for epoch in range(epochs):
            dm.train()
            for m in self._metrics:
                m.reset()
            for step, batch in enumerate(loader):
                if steps_per_epoch is not None and step >= steps_per_epoch:
                    break
                ins, labels = self._split(batch, train_sample_split)
                loss = dm(*ins, *labels)
                history['loss'].append(float(loss))
                if verbose and log_freq and step % log_freq == 0 and (not dist.is_initialized() or dist.get_rank() == 0):
                    print(f"[Engine] epoch {epoch} step {step} loss {history['loss'][-1]:.6f}", flush=True)
            if save_dir is not None and save_freq and (epoch + 1) % save_freq == 0:
                import os
                self.save(os.path.join(save_dir, f'epoch{epoch}'), training=True)
            if valid_data is not None and valid_freq and (epoch + 1) % valid_freq == 0:
                res = self.evaluate(valid_data, valid_sample_split, batch_size, valid_steps, log_freq, collate_fn,
                                    verbose=0)
                for k, v in res.items():
                    history.setdefault('eval_' + k, []).append(v)
        self.history = history
        return history

    def evaluate(self, valid_data, valid_sample_split=None, batch_size=1, steps=None, log_freq=10, collate_fn=None,
                 callbacks=None, verbose=2):
        import torch as _t
        loader = self._loader(valid_data, batch_size, collate_fn)
        self._model.eval()
        for m in self._metrics:
            m.reset()
        losses, res = [], {}
        with _t.no_grad():
            for step, batch in enumerate(loader):
                if steps is not None and step >= steps:
                    break
                ins, labels = self._split(batch, valid_sample_split)
                out = self._model(*ins)
                if self._loss is not None and labels:
                    losses.append(float(self._loss(out, *labels)))
                if self._metrics and labels:
                    res = self._update_metrics(out, labels)
        self._model.train()
        out = {'loss': sum(losses) / len(losses)} if losses else {}
        out.update(res)
        return out

    def predict(self, test_data, test_sample_split=None, batch_size=1, steps=None, collate_fn=None, callbacks=None,
                verbose=2):
        import torch as _t
        loader = self._loader(test_data, batch_size, collate_fn)
        self._model.eval()
        outs = []
        with _t.no_grad():
            for step, batch in enumerate(loader):
                if steps is not None and step >= steps:
                    break
                items = list(batch) if isinstance(batch, (list, tuple)) else [batch]
                k = test_sample_split if test_sample_split is not None else len(items)
                outs.append(self._model(*items[:k]))
        self._model.train()
        return outs

    def run(self, data=None, feed=None, fetch_list=None, mode=None):
        """One step on an already-collated batch ``data`` (inputs..., labels...)."""
        mode = mode or self._mode
        ins, labels = self._split(data, None)
        if mode == 'train':
            return {'loss': float(self._dist_model()(*ins, *labels))}
        import torch as _t
        with _t.no_grad():
            return {'outputs': self._model(*ins)}

    def dataloader(self, dataset, batch_size=1, shuffle=False, drop_last=False, collate_fn=None, num_workers=0,
                   use_buffer_reader=True, use_shared_memory=True, timeout=0, worker_init_fn=None, epochs=1,
                   steps_per_epoch=None, sample_split=1, mode=None):
        return self._loader(dataset, batch_size, collate_fn, shuffle=shuffle)

    def save(self, path, training=True):
        from ....framework.io import save
        save(self._model.state_dict(), path + '.pdparams')
        if training and self._optimizer is not None:
            save(self._optimizer.state_dict(), path + '.pdopt')

    def load(self, path, strict=True, load_optimizer=True):
        import os
        from ....framework.io import load
        self._model.set_state_dict(load(path + '.pdparams'))
        if load_optimizer and self._optimizer is not None and os.path.exists(path + '.pdopt'):
            self._optimizer.set_state_dict(load(path + '.pdopt'))

    def cost(self, inputs_spec=None, labels_spec=None, mode=None):
        return None  # the reference's static cost model; eager steps are timed with paddle.profiler

    @property
    def main_program(self):
        return None

    @property
    def startup_program(self):
        return None

    @property
    def optimizer(self):
        return self._optimizer
