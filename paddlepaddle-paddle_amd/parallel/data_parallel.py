"""Data parallelism with bucketed, backward-overlapped gradient all-reduce over RCCL.

Reference: python/paddle/distributed/parallel.py:202 (DataParallel; coalesced grad groups,
comm_buffer_size / last_comm_buffer_size, find_unused_parameters, no_sync).

MI355X design:
* parameters live in flat buffers (parallel.flat_buffer) — a bucket is just a contiguous slice
  of the flat gradient buffer, so there is no pack/unpack copy before/after the all-reduce;
* buckets are cut in REVERSE registration order (the order backward produces grads), sized
  for xGMI ring bandwidth (default 64 MiB: a few hundred µs per ring all-reduce across 8
  GPUs, big enough to amortise RCCL launch latency, small enough to start early);
* each bucket's all-reduce is launched asynchronously from a post-accumulate-grad hook the
  moment its last gradient lands, so communication of bucket k overlaps the backward
  compute of buckets k+1…; a queued end-of-backward callback flushes partial buckets
  (unused parameters) and makes the compute stream wait on every outstanding collective.
"""
from ..framework.flags import pa_flag  # noqa: E402
import contextlib

import torch
import torch.distributed as dist

from ..core.tensor import Tensor, _wrap, _unwrap
from .flat_buffer import FlatBuffer, register_grad_ready
from ..nn.layer.layers import Layer

DEFAULT_BUCKET_MB = 64


def _pg(group):
    return None if group is None else getattr(group, 'pg', group)


def sync_params_buffers(model, comm_group=None, src_rank=0, is_model_parallel=False, fuse_params=True):
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(_pg(comm_group)) == 1:
        return
    src = src_rank if comm_group is None else comm_group.ranks[src_rank]
    with torch.no_grad():
        tensors = [p._t for p in model.parameters() if not getattr(p, 'is_distributed', False)]
        tensors += [b._t for b in model.buffers()]
        by_dt = {}
        for t in tensors:
            by_dt.setdefault((t.dtype, t.device), []).append(t)
        for ts in by_dt.values():
            flat = torch.cat([t.reshape(-1) for t in ts])
            dist.broadcast(flat, src, group=_pg(comm_group))
            off = 0
            for t in ts:
                n = t.numel()
                t.copy_(flat[off:off + n].view(t.shape))
                off += n


class _Bucket:
    __slots__ = ('buf', 'lo', 'hi', 'params', 'pending', 'work')

    def __init__(self, buf, lo, hi, params):
        self.buf, self.lo, self.hi, self.params = buf, lo, hi, params
        self.pending = len(params)
        self.work = None


class GradAllReducer:
    """Bucketed async all-reduce of flat gradient buffers, driven by autograd hooks."""

    def __init__(self, params, group=None, bucket_mb=DEFAULT_BUCKET_MB, average=True, scale=None,
                 include_distributed=False):
        """average: divide the sum by the group size; scale: multiply the SUM by this factor
        instead (hybrid parallelism reduces over data x sep ranks but averages over data only —
        reference fleet/utils/hybrid_parallel_util.py:241-262); include_distributed: also reduce
        tensor-parallel shards (their data-parallel replicas hold the same shard)."""
        self.group = group
        self.pg = _pg(group)
        self.world = dist.get_world_size(self.pg)
        self.average = average
        self.scale = None if scale is None else float(scale)
        self.enabled = True
        self.buffers = []
        by_dt = {}
        for p in params:
            if p._t.requires_grad and (include_distributed or not getattr(p, 'is_distributed', False)):
                fb = p.__dict__.get('_flat', (None,))[0]
                key = id(fb) if fb is not None else ('new', p._t.dtype)
                by_dt.setdefault(key, []).append(p)
        for key, ps in by_dt.items():
            if isinstance(key, tuple):
                self.buffers.append(FlatBuffer(ps))
            else:
                self.buffers.append(ps[0].__dict__['_flat'][0])
        self.buckets = []
        self._p2b = {}
        cap = int(bucket_mb * 2 ** 20)
        for fb in self.buffers:
            es = fb.grad.element_size()
            hi, cur = fb.numel, []
            for p, o in reversed(list(zip(fb.params, fb.offsets))):
                cur.append(p)
                if (hi - o) * es >= cap:
                    self._add(fb, o, hi, cur)
                    cur, hi = [], o
            if cur:
                self._add(fb, 0, hi, cur)
        self._hooks = []
        for b in self.buckets:
            for p in b.params:
                self._hooks.append(register_grad_ready(p, self._make_hook(b)))
        self._armed = False

    def _add(self, fb, lo, hi, params):
        b = _Bucket(fb, lo, hi, list(params))
        self.buckets.append(b)
        for p in params:
            self._p2b[id(p)] = b
            p.__dict__['_hook_reduced'] = self  # hybrid optimizers skip their own all-reduce of p

    def _make_hook(self, bucket):
        def hook():
            if not self.enabled:
                return
            if not self._armed:
                self._armed = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finish)
            bucket.pending -= 1
            if bucket.pending == 0:
                self._launch(bucket)
        return hook

    def _launch(self, b):
        g = b.buf.grad[b.lo:b.hi]
        if self.scale is None and self.average and dist.get_backend(self.pg) == 'nccl':
            b.work = dist.all_reduce(g, dist.ReduceOp.AVG, group=self.pg, async_op=True)
        else:
            b.work = dist.all_reduce(g, dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def _finish(self):
        from .flat_buffer import run_pre_finish
        run_pre_finish()  # deferred gradient kernels land before any bucket is treated as final
        for b in self.buckets:
            if b.work is None and b.pending != len(b.params):
                self._launch(b)  # partially-touched bucket (unused params): reduce what we have
            elif b.work is None and b.pending == len(b.params):
                self._launch(b)  # untouched bucket: other ranks may have used these params
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                if self.scale is not None:
                    if self.scale != 1.0:
                        b.buf.grad[b.lo:b.hi].mul_(self.scale)
                elif self.average and dist.get_backend(self.pg) != 'nccl':
                    b.buf.grad[b.lo:b.hi].div_(self.world)
            b.work = None
            b.pending = len(b.params)
        self._armed = False

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
        for b in self.buckets:
            for p in b.params:
                if p.__dict__.get('_hook_reduced') is self:
                    del p.__dict__['_hook_reduced']


class DataParallel(Layer):
    """paddle.DataParallel(layers, strategy=None, comm_buffer_size=25, last_comm_buffer_size=1,
    find_unused_parameters=False, group=None)."""

    def __init__(self, layers, strategy=None, comm_buffer_size=DEFAULT_BUCKET_MB, last_comm_buffer_size=1,
                 find_unused_parameters=False, group=None):
        super().__init__()
        self._layers = layers
        self.find_unused_parameters = find_unused_parameters
        self.group = group
        self._strategy = strategy
        import os
        force = pa_flag('force_collectives')  # 1-rank RCCL rehearsal
        ready = dist.is_available() and dist.is_initialized() and (dist.get_world_size(_pg(group)) > 1 or force)
        self._reducer = None
        if ready:
            sync_params_buffers(layers, group)
            self._reducer = GradAllReducer(layers.parameters(), group, max(comm_buffer_size, 1))

    def forward(self, *inputs, **kwargs):
        return self._layers(*inputs, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        r = self._reducer
        prev = r.enabled if r else None
        if r:
            r.enabled = False
        try:
            yield
        finally:
            if r:
                r.enabled = prev

    def scale_loss(self, loss):
        return loss

    def apply_collective_grads(self):
        pass

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layers.set_state_dict(*a, **k)

    set_dict = set_state_dict
    load_dict = set_state_dict
