"""Pipeline parallelism (reference: python/paddle/distributed/fleet/meta_parallel/pipeline_parallel.py:149,
parallel_layers/pp_layers.py: LayerDesc:56, SharedLayerDesc:76, SegmentLayers:92, PipelineLayer:257).

* ``PipelineLayer`` materialises only this stage's slice of the layer list (uniform or
  parameter-balanced segmentation); shared layers (tied embeddings) are replicated on the
  stages that use them and their gradients are all-reduced over the stages sharing them.
* ``PipelineParallel.train_batch`` runs the 1F1B schedule over ``accumulate_steps``
  micro-batches: warm-up forwards, steady 1F1B, cool-down backwards.  Activations and their
  gradients cross stages as point-to-point RCCL send/recv (one xGMI hop on an 8-GPU node);
  tensor metadata (shape/dtype) is exchanged once per batch.
"""
import math

import torch
import torch.distributed as dist

from ....nn.layer.layers import Layer
from ....core.tensor import Tensor, _wrap, _unwrap
from .zero_bubble_utils import WeightGradStore, schedule_order


class LayerDesc:
    def __init__(self, layer_func, *inputs, **kwargs):
        self.layer_func, self.inputs, self.kwargs = layer_func, inputs, kwargs
        if not issubclass(layer_func, Layer):
            raise TypeError("LayerDesc needs a Layer subclass")

    def build_layer(self):
        return self.layer_func(*self.inputs, **self.kwargs)

    def __repr__(self):
        return f"LayerDesc({self.layer_func.__name__})"


class SharedLayerDesc(LayerDesc):
    def __init__(self, key, layer_func, forward_func=None, shared_weight_attr='weight', *inputs, **kwargs):
        super().__init__(layer_func, *inputs, **kwargs)
        self.layer_name = key
        self.forward_func = forward_func
        self.shared_weight_attr = shared_weight_attr


class SegmentLayers:
    def __init__(self, layers_desc, num_parts, method="uniform", num_virtual_pipeline_stage=None):
        self._layers_desc, self.num_parts, self.method = layers_desc, num_parts, method

    def do_segment(self):
        n = len(self._layers_desc)
        if self.method == 'uniform' or not str(self.method).startswith('layer:'):
            base, rem = divmod(n, self.num_parts)
            bounds = [0]
            for i in range(self.num_parts):
                bounds.append(bounds[-1] + base + (1 if i < rem else 0))
            return bounds
        # 'layer:ClassName' → balance the count of that layer type across stages
        name = self.method.split(':', 1)[1]
        idx = [i for i, d in enumerate(self._layers_desc)
               if (d.layer_func.__name__ if isinstance(d, LayerDesc) else type(d).__name__) == name]
        per = math.ceil(len(idx) / self.num_parts)
        bounds = [0]
        for s in range(1, self.num_parts):
            k = min(s * per, len(idx) - 1)
            bounds.append(idx[k] if k < len(idx) else n)
        bounds.append(n)
        return bounds


class PipelineLayer(Layer):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seg_method="uniform",
                 recompute_interval=0, recompute_ctx=None, num_virtual_pipeline_stages=None):
        super().__init__()
        from ... import fleet as _fleet
        hcg = _fleet.get_hybrid_communicate_group() if _fleet._inited() else None
        self._num_stages = num_stages or (hcg.get_pipe_parallel_world_size() if hcg else 1)
        self._stage_id = hcg.get_stage_id() if hcg else 0
        self._hcg = hcg
        self._loss_fn = loss_fn
        self._recompute_interval = recompute_interval
        self._layers_desc = list(layers)
        self._num_virtual = int(num_virtual_pipeline_stages or 1)
        nparts = self._num_stages * self._num_virtual
        self.segment_parts = SegmentLayers(self._layers_desc, nparts, seg_method).do_segment()
        # virtual stage k of this rank is global chunk (k * num_stages + stage_id)
        self._chunk_ranges = [(self.segment_parts[k * self._num_stages + self._stage_id],
                               self.segment_parts[k * self._num_stages + self._stage_id + 1])
                              for k in range(self._num_virtual)]
        lo, hi = self._chunk_ranges[0]
        self._start, self._end = lo, hi
        self.run_function = []
        self._chunks = []
        from ....nn.layer.container import LayerDict, LayerList
        self.shared_layers = LayerDict()  # registered: the optimizer sees the shared weights
        self._shared_descs = {}
        built = []
        for lo_k, hi_k in self._chunk_ranges:
            start = len(self.run_function)
            self._build_range(lo_k, hi_k, built)
            self._chunks.append(self.run_function[start:])
        self.layers = LayerList(built)
        self._shared_names = list(self.shared_layers.keys())
        self._shared_comm = self._build_shared_comm()

    def _build_range(self, lo, hi, built):
        for i, d in enumerate(self._layers_desc[lo:hi]):
            if isinstance(d, SharedLayerDesc):
                if d.layer_name not in self.shared_layers:
                    self.shared_layers[d.layer_name] = d.build_layer()
                    self._shared_descs[d.layer_name] = d
                layer = self.shared_layers[d.layer_name]
                fn = (lambda l, f: (lambda x: f(l, x)))(layer, d.forward_func) if d.forward_func else layer
                self.run_function.append(fn)
            elif isinstance(d, LayerDesc):
                layer = d.build_layer()
                built.append(layer)
                self.run_function.append(layer)
            elif isinstance(d, Layer):
                built.append(d)
                self.run_function.append(d)
            else:
                self.run_function.append(d)

    def get_num_virtual_stages(self):
        return self._num_virtual

    def _build_shared_comm(self):
        """Groups of stages that hold a copy of each shared layer (for grad all-reduce)."""
        comm = {}
        if self._num_stages == 1 or not dist.is_initialized():
            return comm
        keys = {}
        for part in range(len(self.segment_parts) - 1):
            s = part % self._num_stages
            lo, hi = self.segment_parts[part], self.segment_parts[part + 1]
            for d in self._layers_desc[lo:hi]:
                if isinstance(d, SharedLayerDesc):
                    keys.setdefault(d.layer_name, set()).add(s)
        from ...communication import new_group
        for k, stages in sorted(keys.items()):
            stages = sorted(stages)
            if len(stages) < 2:
                continue
            # one group per pipeline replica (every rank creates every group, in the same order)
            me = dist.get_rank()
            for pipe_ranks in self._hcg.topology().get_comm_list('pipe'):
                ranks = [pipe_ranks[s] for s in stages]
                g_ = new_group(ranks)
                if me in ranks:
                    g = g_
            if self._stage_id in stages:
                ranks = [self._hcg.get_rank_from_stage(s) for s in stages]
                comm[k] = g
                for p in self.shared_layers[k].parameters():
                    # (key, counted elsewhere): a sharding optimizer gives these their own unit so
                    # the stages' shards line up, and global-norm clipping counts them on one stage
                    p.__dict__['_pp_shared'] = (k, self._stage_id != stages[0])
                    with torch.no_grad():  # every copy starts from the first holder's weights
                        dist.broadcast(p._t, ranks[0], group=g.pg)
        return comm

    def allreduce_shared_weight_gradients(self):
        for k, g in self._shared_comm.items():
            for p in self.shared_layers[k].parameters():
                if p._t.grad is not None:
                    dist.all_reduce(p._t.grad, group=g.pg)

    def get_stage_from_index(self, layer_idx):
        for s in range(self._num_stages):
            if self.segment_parts[s] <= layer_idx < self.segment_parts[s + 1]:
                return s
        return self._num_stages - 1

    def forward(self, input, chunk_id=None):  # noqa: A002
        x = input
        funcs = self._chunks[chunk_id] if chunk_id is not None else self.run_function
        for i, f in enumerate(funcs):
            if self._recompute_interval and self.training and i % self._recompute_interval == 0 and \
                    isinstance(f, Layer) and any(not p.stop_gradient for p in f.parameters()):
                from ..recompute import recompute
                x = recompute(f, *(x if isinstance(x, tuple) else (x,)))
            else:
                x = f(*x) if isinstance(x, tuple) else f(x)
        return x


class PipelineParallel(Layer):
    """Wraps a PipelineLayer; ``train_batch`` runs 1F1B over micro-batches."""

    def __init__(self, layers, hcg, strategy):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        cfg = getattr(strategy, 'pipeline_configs', {}) or {}
        self.accumulate_steps = int(cfg.get('accumulate_steps', 1))
        self.micro_batch_size = cfg.get('micro_batch_size', None)
        self.num_stages = hcg.get_pipe_parallel_world_size()
        self.stage_id = hcg.get_stage_id()
        self.pp_group = hcg.get_pipe_parallel_group()
        self.is_first = self.stage_id == 0
        self.is_last = self.stage_id == self.num_stages - 1
        self._prev = hcg.prev_rank
        self._next = hcg.next_rank
        # gradients sync over dp, or dp x sep when the sequence is also split (reference
        # pipeline_parallel.py:185-187); replicas start from the same weights
        from ..utils.hybrid_parallel_util import (dp_sep_group_and_scale, broadcast_dp_parameters,
                                                  broadcast_sep_parameters)
        self._dp_group = dp_sep_group_and_scale(hcg)[0]
        # 'schedule_mode': '1F1B' (default) or 'ZBH1' (zero bubble, reference
        # passes/pipeline_scheduler_pass/pipeline_zero_bubble.py)
        self._schedule_mode = cfg.get('schedule_mode', '1F1B')
        if hcg.get_sep_parallel_world_size() > 1:
            broadcast_sep_parameters(self._layers, hcg)
        if hcg.get_data_parallel_world_size() > 1 and hcg.get_sharding_parallel_world_size() == 1:
            broadcast_dp_parameters(self._layers, hcg)
        self._meta_fwd = None
        self._meta_bwd = None
        self.total_loss = None
        self._sends = []
        # gradients travel on a second pipe communicator: each (src, dst) channel then carries ONE
        # kind of message in schedule order, so receives can be posted ahead of the compute that
        # precedes them without ever being matched against the wrong send (on RCCL every pair
        # communicator is one stream: a pre-posted activation receive must not sit in front of a
        # gradient send the peer is waiting for).  Every rank creates every pipe group, in order.
        self._grad_pg = None
        topo = hcg.topology()
        if self.num_stages > 1:
            for ranks in topo.get_comm_list('pipe'):
                g = hcg._mk(ranks)
                if hcg.global_rank in ranks:
                    self._grad_pg = g
        self._act_q = []   # posted (work, buffer) activation receives, in micro-batch order
        self._grad_q = []  # posted (work, buffer) gradient receives
        self._acts_left = 0
        self._grads_left = 0
        self._meta_bwd = None

    def forward(self, *a, **k):
        return self._layers(*a, **k)

    # ---- p2p helpers (metadata once per batch, then raw tensors; receives posted ahead)
    def _gpg(self):
        return None if self._grad_pg is None else getattr(self._grad_pg, 'pg', None)

    def _send_meta(self, t, peer):
        meta = torch.tensor([len(t.shape)] + list(t.shape) + [_DT.index(t.dtype)], dtype=torch.int64)
        meta = meta.to(t.device)
        n = torch.tensor([meta.numel()], dtype=torch.int64, device=t.device)
        self._isend(n, peer)
        self._isend(meta, peer)

    def _isend(self, t, peer, group=None):
        """Sends never block the schedule: in steady 1F1B a stage sends an activation forward
        while its neighbour sends a gradient back, so blocking sends would deadlock."""
        self._sends.append((dist.isend(t, peer, group=group), t))

    def _drain_sends(self):
        for w, _ in self._sends:
            w.wait()
        self._sends = []

    def _recv_meta(self, peer, dev):
        n = torch.empty(1, dtype=torch.int64, device=dev)
        dist.recv(n, peer)
        meta = torch.empty(int(n.item()), dtype=torch.int64, device=dev)
        dist.recv(meta, peer)
        m = meta.tolist()
        nd = m[0]
        return tuple(m[1:1 + nd]), _DT[m[1 + nd]]

    def _post_act(self, dev):
        """Posts the receive of the next expected activation (it lands while this stage computes)."""
        if self._acts_left > 0:
            shape, dt = self._meta_fwd
            buf = torch.empty(shape, dtype=dt, device=dev)
            self._act_q.append((dist.irecv(buf, self._prev), buf))
            self._acts_left -= 1

    def _post_grad(self, dev):
        if self._grads_left > 0 and self._meta_bwd is not None:
            shape, dt = self._meta_bwd
            buf = torch.empty(shape, dtype=dt, device=dev)
            self._grad_q.append((dist.irecv(buf, self._next, group=self._gpg()), buf))
            self._grads_left -= 1

    @staticmethod
    def _take(q):
        w, buf = q.pop(0)
        w.wait()  # RCCL: the compute stream waits on the receive; the host does not block
        return buf

    def _dev(self):
        return torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() else torch.device('cpu')

    def _split(self, data):
        if isinstance(data, (list, tuple)):
            parts = [self._split(d) for d in data]
            return [tuple(p[i] for p in parts) for i in range(self.accumulate_steps)]
        t = _unwrap(data)
        return [_wrap(c) for c in t.chunk(self.accumulate_steps, 0)]

    def _begin(self, n_fwd, n_bwd):
        self._sent_meta = False
        self._meta_fwd = None
        self._meta_bwd = None
        self._act_q, self._grad_q = [], []
        self._acts_left = 0 if self.is_first else n_fwd
        self._grads_left = 0 if self.is_last else n_bwd

    def _fwd_step(self, mb_input, mb_label):
        dev = self._dev()
        if self.is_first:
            x = mb_input
        else:
            if self._meta_fwd is None:
                self._meta_fwd = self._recv_meta(self._prev, dev)
                self._post_act(dev)
            buf = self._take(self._act_q)
            self._post_act(dev)  # prefetch the next micro-batch's activation under this compute
            buf.requires_grad_(True)
            x = _wrap(buf)
        out = self._layers(x)
        if self.is_last:
            loss = self._layers._loss_fn(out, mb_label) if self._layers._loss_fn is not None else out
            loss = _wrap(_unwrap(loss) / self.accumulate_steps)
            return x, loss
        o = _unwrap(out)
        if not self._sent_meta:
            self._send_meta(o, self._next)
            self._sent_meta = True
        self._isend(o.detach().contiguous(), self._next)
        if self._meta_bwd is None and self._grads_left > 0:
            # the gradient of this stage's output has the output's shape: post its receive now
            self._meta_bwd = (tuple(o.shape), o.dtype)
            self._post_grad(dev)
        return x, out

    def _set_dp_final(self, optimizer, final):
        eng = getattr(optimizer, 'engine', None)
        if eng is not None and hasattr(eng, 'dp_final'):
            eng.dp_final = bool(final)

    def _bwd_step(self, x, out, split=False):
        """Backward of one micro-batch; ``split`` (zero bubble): only B runs here — the Linear
        weight gradients are queued in the WeightGradStore and run by _w_step after the input
        gradient has been sent."""
        if self.is_last:
            _unwrap(out).backward()
        else:
            o = _unwrap(out)
            g = self._take(self._grad_q)
            self._post_grad(o.device)
            o.backward(g)
        if split:
            WeightGradStore.flush()
        if not self.is_first:
            gx = _unwrap(x).grad
            self._isend(gx.contiguous(), self._prev, group=self._gpg())

    def _w_step(self):
        WeightGradStore.pop()

    def _schedule_kind(self, optimizer):
        kind = str(self._schedule_mode or '1F1B').upper().replace('-', '')
        if kind in ('ZBH1', 'ZB', 'ZEROBUBBLE'):
            if getattr(optimizer, '_syncs_dp', False):
                # a sharding optimizer reduce-scatters inside backward: its gradient hooks must see
                # complete weight gradients, which only the unsplit backward gives
                import warnings
                warnings.warn("ZBH1 pipeline schedule with a sharding optimizer: running 1F1B", RuntimeWarning)
                return '1F1B'
            return 'ZBH1'
        return '1F1B'

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        inputs, labels = data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
        mbs_in = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
        mbs_lab = self._split(labels) if (self.is_last and labels is not None) else [None] * self.accumulate_steps
        n = self.accumulate_steps
        self._begin(n, n)
        kind = self._schedule_kind(optimizer)
        split = kind == 'ZBH1'
        # the stage's op sequence (zero_bubble_utils.schedule_order: 1F1B, or ZB-H1 with every
        # backward split into B — input gradient, sent at once — and W — weight gradients)
        pending, losses = {}, []
        WeightGradStore.clear()
        WeightGradStore.active = split
        try:
            for op, i in schedule_order(kind, self.num_stages, self.stage_id, n):
                if op == 'F':
                    x, out = self._fwd_step(mbs_in[i], mbs_lab[i])
                    pending[i] = (x, out)
                    if self.is_last:
                        losses.append(_unwrap(out).detach())
                elif op in ('B', 'BW'):
                    self._set_dp_final(optimizer, i == n - 1)  # dp all-reduce overlap on the last micro-batch
                    self._bwd_step(*pending.pop(i), split=split)
                else:
                    self._w_step()
        finally:
            WeightGradStore.active = False
        assert not pending and WeightGradStore.pending() == 0
        self._set_dp_final(optimizer, True)
        assert not (self._act_q or self._grad_q or self._acts_left or self._grads_left), "unmatched pipeline receives"
        self._drain_sends()
        if getattr(optimizer, '_syncs_dp', False):
            # the sharding optimizer reduce-scattered the gradients inside backward: sum the shared
            # weights' shards (own units, identical slicing on every holder) over their stages
            optimizer._sync_shared_grads(self._layers._shared_comm)
        else:
            self._layers.allreduce_shared_weight_gradients()
        if self._dp_group is not None and self._dp_group.nranks > 1 and not getattr(optimizer, '_syncs_dp', False):
            # one coalesced all-reduce per dtype (a sharding optimizer syncs dp on its shards instead)
            from ..utils.hybrid_parallel_util import fused_allreduce_gradients
            fused_allreduce_gradients(list(self._layers.parameters()), self._hcg)
        if scaler is not None:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
        optimizer.clear_grad()
        if lr_scheduler is not None:
            lr_scheduler.step()
        # broadcast the mean loss from the last stage to every stage
        dev = self._dev()
        loss = torch.stack(losses).sum() if self.is_last else torch.zeros((), device=dev)
        loss = loss.to(dev).float()
        if self.num_stages > 1:
            dist.broadcast(loss, self._hcg.get_rank_from_stage(self.num_stages - 1), group=self.pp_group.pg)
        self.total_loss = _wrap(loss)
        return self.total_loss

    def eval_batch(self, data, compute_loss=True):
        with torch.no_grad():
            inputs, labels = data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
            mbs_in = self._split(inputs) if self.is_first else [None] * self.accumulate_steps
            mbs_lab = self._split(labels) if (self.is_last and labels is not None) else [None] * self.accumulate_steps
            self._begin(self.accumulate_steps, 0)
            outs = []
            for i in range(self.accumulate_steps):
                _, out = self._fwd_step(mbs_in[i], mbs_lab[i])
                if self.is_last:
                    outs.append(_unwrap(out))
            self._drain_sends()
            if self.is_last:
                return _wrap(torch.stack(outs).sum() if compute_loss else torch.cat(outs))
            return None


class PipelineParallelWithInterleave(PipelineParallel):
    """Virtual pipeline stages (reference: pipeline_parallel.py PipelineParallelWithInterleave):
    rank r holds global chunks r, r+P, r+2P, ...; activations travel rank 0 → P-1 and wrap to
    rank 0's next chunk.

    Schedule: interleaved 1F1B (warm-up of 2(P-r-1) + (V-1)P forward units, then alternating
    one forward / one backward unit, then the backward cool-down), the schedule of the reference's
    interleaved pipeline; unit k runs micro-batch ``(k // PV) P + k % P`` through chunk
    ``(k % PV) // P`` (reversed for backward).  Needs accumulate_steps % P == 0 (as the reference
    does); otherwise the breadth-first order (every micro-batch through chunk 0, then chunk 1, …)
    runs instead.  Activations and gradients travel on two communicators, so each (src, dst) channel
    carries one kind of message in one global order: sends are asynchronous, receives block, and
    the schedule is deadlock-free for every P, V (checked by simulation and the gloo tests)."""

    def __init__(self, layers, hcg, strategy):
        super().__init__(layers, hcg, strategy)  # creates the gradient communicator
        self.schedule = 'interleaved_1f1b'

    def _peer(self, delta):
        s = (self.stage_id + delta) % self.num_stages
        return self._hcg.get_rank_from_stage(s)

    def _pg_of(self, kind):
        g = self._grad_pg if kind == 'grad' else self.pp_group
        return None if g is None else getattr(g, 'pg', None)

    def _send(self, t, peer, kind='act'):
        pg = self._pg_of(kind)
        t = t.detach().contiguous()
        meta = torch.tensor([len(t.shape)] + list(t.shape) + [_DT.index(t.dtype)], dtype=torch.int64, device=t.device)
        n = torch.tensor([meta.numel()], dtype=torch.int64, device=t.device)
        for x in (n, meta, t):
            self._sends.append((dist.isend(x, peer, group=pg), x))

    def _recv(self, peer, dev, kind='act'):
        pg = self._pg_of(kind)
        n = torch.empty(1, dtype=torch.int64, device=dev)
        dist.recv(n, peer, group=pg)
        meta = torch.empty(int(n.item()), dtype=torch.int64, device=dev)
        dist.recv(meta, peer, group=pg)
        m = meta.tolist()
        nd = m[0]
        buf = torch.empty(tuple(m[1:1 + nd]), dtype=_DT[m[1 + nd]], device=dev)
        dist.recv(buf, peer, group=pg)
        return buf

    def _units(self, n, V, P, r):
        """The rank's ordered list of ('F' | 'B', chunk, micro-batch) units."""
        if V == 1 or n % P != 0:
            self.schedule = 'breadth_first'
            return ([('F', v, m) for v in range(V) for m in range(n)] +
                    [('B', v, m) for v in reversed(range(V)) for m in range(n)])
        self.schedule = 'interleaved_1f1b'
        from .zero_bubble_utils import interleaved_units
        return interleaved_units(n, V, P, r)

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None):
        inputs, labels = data if isinstance(data, (list, tuple)) and len(data) == 2 else (data, None)
        n, V, P = self.accumulate_steps, self._layers.get_num_virtual_stages(), self.num_stages
        first_rank, last_rank = self.is_first, self.is_last
        mbs_in = self._split(inputs) if first_rank else [None] * n
        mbs_lab = self._split(labels) if (last_rank and labels is not None) else [None] * n
        dev = self._dev()
        prev_rank, next_rank = self._peer(-1), self._peer(+1)
        saved = {}
        losses = {}
        for kind, v, m in self._units(n, V, P, self.stage_id):
            if kind == 'F':
                if first_rank and v == 0:
                    x = mbs_in[m]
                else:
                    buf = self._recv(prev_rank, dev, 'act')
                    buf.requires_grad_(True)
                    x = _wrap(buf)
                out = self._layers(x, chunk_id=v)
                if last_rank and v == V - 1:
                    loss = self._layers._loss_fn(out, mbs_lab[m]) if self._layers._loss_fn is not None else out
                    loss = _wrap(_unwrap(loss) / n)
                    losses[m] = _unwrap(loss).detach()
                    saved[(v, m)] = (x, loss)
                else:
                    self._send(_unwrap(out), next_rank, 'act')
                    saved[(v, m)] = (x, out)
            else:
                x, out = saved.pop((v, m))
                if last_rank and v == V - 1:
                    _unwrap(out).backward()
                else:
                    g = self._recv(next_rank, dev, 'grad')
                    _unwrap(out).backward(g)
                if not (first_rank and v == 0):
                    self._send(_unwrap(x).grad, prev_rank, 'grad')
        self._drain_sends()
        if getattr(optimizer, '_syncs_dp', False):
            # the sharding optimizer reduce-scattered the gradients inside backward: sum the shared
            # weights' shards (own units, identical slicing on every holder) over their stages
            optimizer._sync_shared_grads(self._layers._shared_comm)
        else:
            self._layers.allreduce_shared_weight_gradients()
        if self._dp_group is not None and self._dp_group.nranks > 1 and not getattr(optimizer, '_syncs_dp', False):
            # one coalesced all-reduce per dtype (a sharding optimizer syncs dp on its shards instead)
            from ..utils.hybrid_parallel_util import fused_allreduce_gradients
            fused_allreduce_gradients(list(self._layers.parameters()), self._hcg)
        if scaler is not None:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
        optimizer.clear_grad()
        if lr_scheduler is not None:
            lr_scheduler.step()
        loss = torch.stack([losses[m] for m in sorted(losses)]).sum() if last_rank else torch.zeros((), device=dev)
        loss = loss.to(dev).float()
        if P > 1:
            dist.broadcast(loss, self._hcg.get_rank_from_stage(P - 1), group=self.pp_group.pg)
        self.total_loss = _wrap(loss)
        return self.total_loss



class PipelineParallelWithInterleaveFthenB(PipelineParallelWithInterleave):
    """Virtual pipeline stages with the forward-then-backward order (reference:
    pipeline_parallel.py:1831 PipelineParallelWithInterleaveFthenB; fleet.distributed_model picks
    it when pp_degree <= accumulate_steps < 2 * pp_degree): every forward unit of the interleaved
    order first, then every backward unit in reverse — the interleaved 1F1B schedule without its
    steady state, which needs fewer micro-batches (P) than 1F1B's warm-up (2P) at the cost of
    holding all micro-batches' activations.  Sends are asynchronous and receives block in one
    global order per channel, so the schedule is deadlock-free like the 1F1B one."""

    def _units(self, n, V, P, r):
        total = n * V
        fch = lambda k: (k % (P * V)) // P  # noqa: E731
        mb = lambda k: (k // (P * V)) * P + k % P  # noqa: E731
        if n % P != 0:
            self.schedule = 'breadth_first'
            return ([('F', v, m) for v in range(V) for m in range(n)] +
                    [('B', v, m) for v in reversed(range(V)) for m in range(n)])
        self.schedule = 'interleaved_fthenb'
        return ([('F', fch(k), mb(k)) for k in range(total)] +
                [('B', V - 1 - fch(k), mb(k)) for k in range(total)])

_DT = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.bool]
