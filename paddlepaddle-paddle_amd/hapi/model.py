"""High-level Model API (reference: python/paddle/hapi/model.py — Model:1052 prepare:1670,
fit:1750, evaluate:1999, predict:2110, save:1356, load:1423, train_batch:1194, summary:2376;
DynamicGraphAdapter:776).

One process per GPU: when launched with WORLD_SIZE>1 the network is wrapped in our
bucketed DataParallel and loaders get a DistributedBatchSampler automatically.
"""
import os

import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap
from ..io import DataLoader, Dataset, DistributedBatchSampler
from ..metric import Metric
from .callbacks import config_callbacks


def to_list(value):
    if value is None:
        return []
    if isinstance(value, (list, tuple)):
        return list(value)
    return [value]


def _to_np(v):
    if isinstance(v, Tensor):
        t = v._t.detach()
        return (t.float() if t.dtype == torch.bfloat16 else t).cpu().numpy()
    return np.asarray(v)


class Model:
    def __init__(self, network, inputs=None, labels=None):
        self.network = network
        self._inputs = to_list(inputs)
        self._labels = to_list(labels)
        self._loss = None
        self._optimizer = None
        self._metrics = []
        self._amp_level = 'O0'
        self._amp_dtype = 'float16'
        self._scaler = None
        self.stop_training = False
        self._world = int(os.environ.get('WORLD_SIZE', '1'))
        self._dp = None
        self._accumulate = 1
        self._acc_step = 0

    # ---- setup
    def prepare(self, optimizer=None, loss=None, metrics=None, amp_configs=None):
        self._optimizer = optimizer
        self._loss = loss
        self._metrics = to_list(metrics)
        for m in self._metrics:
            if not isinstance(m, Metric):
                raise TypeError(f"{type(m).__name__} is not a paddle.metric.Metric")
        if amp_configs is not None:
            cfg = {'level': amp_configs} if isinstance(amp_configs, str) else dict(amp_configs)
            self._amp_level = cfg.get('level', 'O1')
            self._amp_dtype = cfg.get('dtype', 'bfloat16')
            if self._amp_level in ('O1', 'O2') and self._amp_dtype == 'float16':
                from ..amp import GradScaler
                self._scaler = GradScaler(init_loss_scaling=cfg.get('init_loss_scaling', 2.0 ** 15))
            if self._amp_level == 'O2' and optimizer is not None:
                from .. import amp
                self.network, self._optimizer = amp.decorate(self.network, optimizer, level='O2',
                                                             dtype=self._amp_dtype)
        if self._world > 1 and self._dp is None:
            from .. import distributed as dist
            if not dist.is_initialized():
                dist.init_parallel_env()
            from ..parallel.data_parallel import DataParallel
            self._dp = DataParallel(self.network)

    def _net(self):
        return self._dp if self._dp is not None else self.network

    def parameters(self, *args, **kwargs):
        return self.network.parameters(*args, **kwargs)

    # ---- batch steps
    def _forward(self, inputs):
        from .. import amp
        if self._amp_level in ('O1', 'O2'):
            with amp.auto_cast(level=self._amp_level, dtype=self._amp_dtype):
                return self._net()(*inputs)
        return self._net()(*inputs)

    def _compute_loss(self, outputs, labels):
        outs = to_list(outputs)
        if self._loss is None:
            return outs[0] if outs else None
        losses = to_list(self._loss(*(outs + labels)))
        total = losses[0]
        for l_ in losses[1:]:
            total = total + l_
        return total, losses

    def _update_metrics(self, outputs, labels):
        res = []
        for m in self._metrics:
            st = m.compute(*(to_list(outputs) + labels))
            res.append(m.update(*[_to_np(s) for s in to_list(st)]))
        return res

    def train_batch(self, inputs, labels=None, update=True):
        self.network.train()
        inputs, labels = [_as_t(x) for x in to_list(inputs)], [_as_t(x) for x in to_list(labels)]
        outputs = self._forward(inputs)
        total, losses = self._compute_loss(outputs, labels)
        scaled = total / self._accumulate if self._accumulate > 1 else total
        if self._scaler is not None:
            self._scaler.scale(scaled).backward()
        else:
            scaled.backward()
        if update:
            if self._scaler is not None:
                self._scaler.minimize(self._optimizer, scaled)
            else:
                self._optimizer.step()
            self._optimizer.clear_grad()
        metrics = self._update_metrics(outputs, labels)
        loss_np = [float(_to_np(l_)) for l_ in losses]
        return (loss_np, metrics) if self._metrics else loss_np

    @torch.no_grad()
    def eval_batch(self, inputs, labels=None):
        self.network.eval()
        inputs, labels = [_as_t(x) for x in to_list(inputs)], [_as_t(x) for x in to_list(labels)]
        outputs = self._forward(inputs)
        loss_np = []
        if self._loss is not None and labels:
            _, losses = self._compute_loss(outputs, labels)
            loss_np = [float(_to_np(l_)) for l_ in losses]
        metrics = self._update_metrics(outputs, labels)
        return (loss_np, metrics) if self._metrics else loss_np

    @torch.no_grad()
    def predict_batch(self, inputs):
        self.network.eval()
        outputs = self._forward([_as_t(x) for x in to_list(inputs)])
        return [_to_np(o) for o in to_list(outputs)]

    # ---- loops
    def _loader(self, data, batch_size, shuffle, drop_last, num_workers):
        if data is None or isinstance(data, DataLoader):
            return data
        if isinstance(data, Dataset):
            if self._world > 1:
                bs = DistributedBatchSampler(data, batch_size, shuffle=shuffle, drop_last=drop_last)
                return DataLoader(data, batch_sampler=bs, num_workers=num_workers)
            return DataLoader(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last,
                              num_workers=num_workers)
        return data  # any iterable of batches

    def _split(self, batch):
        batch = to_list(batch)
        n_in = len(self._inputs) if self._inputs else max(len(batch) - (len(self._labels) or 1), 1)
        if not self._labels and self._loss is None and not self._metrics:
            n_in = len(batch)
        return batch[:n_in], batch[n_in:]

    def _logs(self, res, prefix=''):
        logs = {}
        if self._metrics:
            losses, metrics = res
        else:
            losses, metrics = res, []
        if losses:
            logs[prefix + 'loss'] = losses[0] if len(losses) == 1 else losses
        for m, v in zip(self._metrics, metrics):
            names = m.name() if isinstance(m.name(), list) else [m.name()]
            vals = v if isinstance(v, (list, tuple)) else [v]
            for n, x in zip(names, vals):
                logs[prefix + n] = x
        return logs

    def fit(self, train_data=None, eval_data=None, batch_size=1, epochs=1, eval_freq=1, log_freq=10, save_dir=None,
            save_freq=1, verbose=2, drop_last=False, shuffle=True, num_workers=0, callbacks=None,
            accumulate_grad_batches=1, num_iters=None):
        if self._optimizer is None or self._loss is None:
            raise RuntimeError("call prepare(optimizer, loss) before fit")
        train_loader = self._loader(train_data, batch_size, shuffle, drop_last, num_workers)
        eval_loader = self._loader(eval_data, batch_size, False, False, num_workers)
        self._accumulate = max(1, accumulate_grad_batches)
        try:
            steps = len(train_loader)
        except (TypeError, ValueError):
            steps = None
        metric_names = []
        for m in self._metrics:
            metric_names += to_list(m.name())
        cbks = config_callbacks(callbacks, model=self, batch_size=batch_size, epochs=epochs, steps=steps,
                                log_freq=log_freq, verbose=verbose, save_freq=save_freq, save_dir=save_dir,
                                metrics=metric_names)
        cbks.params['save_dir'] = save_dir
        self.stop_training = False
        cbks.on_begin('train')
        it_count = 0
        for epoch in range(epochs):
            for m in self._metrics:
                m.reset()
            cbks.on_epoch_begin(epoch)
            logs = {}
            for step, batch in enumerate(train_loader):
                cbks.on_batch_begin('train', step, logs)
                ins, labs = self._split(batch)
                update = (step + 1) % self._accumulate == 0 or (steps is not None and step + 1 == steps)
                res = self.train_batch(ins, labs, update=update)
                logs = self._logs(res)
                logs['batch_size'] = _batch_len(ins)
                cbks.on_batch_end('train', step, logs)
                it_count += 1
                if num_iters is not None and it_count >= num_iters:
                    self.stop_training = True
                    break
            for m in self._metrics:
                acc = m.accumulate()
                names = to_list(m.name())
                for n, v in zip(names, to_list(acc)):
                    logs[n] = v
            cbks.on_epoch_end(epoch, logs)
            if eval_loader is not None and (epoch + 1) % eval_freq == 0:
                self._run_eval(eval_loader, cbks, log_freq)
            if self.stop_training:
                break
        cbks.on_end('train', logs)

    def _run_eval(self, loader, cbks, log_freq=10, num_iters=None):
        for m in self._metrics:
            m.reset()
        cbks.on_begin('eval')
        losses = []
        n = 0
        for step, batch in enumerate(loader):
            cbks.on_batch_begin('eval', step)
            ins, labs = self._split(batch)
            res = self.eval_batch(ins, labs)
            l_ = res[0] if self._metrics else res
            if l_:
                losses.append(l_[0])
            n += _batch_len(ins)
            cbks.on_batch_end('eval', step, self._logs(res))
            if num_iters is not None and step + 1 >= num_iters:
                break
        logs = {}
        if losses:
            logs['loss'] = [float(np.mean(losses))]
        for m in self._metrics:
            for k, v in zip(to_list(m.name()), to_list(m.accumulate())):
                logs[k] = v
        logs['batch_size'] = n
        cbks.on_end('eval', logs)
        return logs

    def evaluate(self, eval_data, batch_size=1, log_freq=10, verbose=2, num_workers=0, callbacks=None,
                 num_iters=None):
        loader = self._loader(eval_data, batch_size, False, False, num_workers)
        cbks = config_callbacks(callbacks, model=self, batch_size=batch_size, log_freq=log_freq, verbose=verbose,
                                metrics=[n for m in self._metrics for n in to_list(m.name())], mode='eval')
        logs = self._run_eval(loader, cbks, log_freq, num_iters)
        logs.pop('batch_size', None)
        return logs

    def predict(self, test_data, batch_size=1, num_workers=0, stack_outputs=False, verbose=1, callbacks=None):
        loader = self._loader(test_data, batch_size, False, False, num_workers)
        cbks = config_callbacks(callbacks, model=self, batch_size=batch_size, verbose=verbose, mode='test')
        cbks.on_begin('predict')
        outs = []
        for step, batch in enumerate(loader):
            ins = to_list(batch)
            if self._inputs:
                ins = ins[:len(self._inputs)]
            outs.append(self.predict_batch(ins))
            cbks.on_batch_end('predict', step)
        cbks.on_end('predict')
        res = list(zip(*outs))
        if stack_outputs:
            res = [np.concatenate(r, 0) for r in res]
        else:
            res = [list(r) for r in res]
        return res

    # ---- persistence
    def save(self, path, training=True):
        from ..framework.io import save as psave
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if training:
            psave(self.network.state_dict(), path + '.pdparams')
            if self._optimizer is not None:
                psave(self._optimizer.state_dict(), path + '.pdopt')
        else:
            from .. import jit
            specs = self._inputs or None
            jit.save(self.network, path, input_spec=specs)

    def load(self, path, skip_mismatch=False, reset_optimizer=False):
        from ..framework.io import load as pload
        p = path if path.endswith('.pdparams') else path + '.pdparams'
        state = pload(p)
        if skip_mismatch:
            own = self.network.state_dict()
            state = {k: v for k, v in state.items() if k in own and list(own[k].shape) == list(v.shape)}
        self.network.set_state_dict(state)
        opt_path = p[:-len('.pdparams')] + '.pdopt'
        if not reset_optimizer and self._optimizer is not None and os.path.exists(opt_path):
            self._optimizer.set_state_dict(pload(opt_path))

    def summary(self, input_size=None, dtype=None):
        from .model_summary import summary
        if input_size is None and self._inputs:
            input_size = [tuple(s.shape) for s in self._inputs]
        return summary(self.network, input_size, dtype)


def _as_t(x):
    if isinstance(x, Tensor):
        return x
    from ..core.tensor import to_tensor
    return to_tensor(x)


def _batch_len(ins):
    for x in ins:
        if hasattr(x, 'shape') and len(x.shape) > 0:
            return x.shape[0]
    return 1
