"""Tensor-parallel communication primitives as autograd functions
(reference: python/paddle/distributed/fleet/layers/mpu/mp_ops.py: c_identity, c_split, c_concat,
mp_allreduce, c_softmax_with_cross_entropy).

All run on the model-parallel RCCL communicator; with mp degree 1 they are identities.
"""
import torch
import torch.distributed as dist

from .....core.tensor import Tensor, _wrap, _unwrap


def _pg(group):
    return None if group is None else getattr(group, 'pg', group)


def _n(group):
    if group is None or not dist.is_initialized():
        return 1
    return group.nranks if hasattr(group, 'nranks') else dist.get_world_size(_pg(group))


def _r(group):
    if group is None or not dist.is_initialized():
        return 0
    return group.rank if hasattr(group, 'rank') else dist.get_rank(_pg(group))


class _Identity(torch.autograd.Function):
    """fwd: identity; bwd: all-reduce (entry of a column-parallel region)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if _n(ctx.group) > 1:
            g = g.contiguous()
            dist.all_reduce(g, group=_pg(ctx.group))
        return g, None


class _AllReduce(torch.autograd.Function):
    """fwd: all-reduce; bwd: identity (exit of a row-parallel region)."""

    @staticmethod
    def forward(ctx, x, group):
        if _n(group) > 1:
            x = x.contiguous().clone()
            dist.all_reduce(x, group=_pg(group))
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _Split(torch.autograd.Function):
    """fwd: keep this rank's slice of the last dim; bwd: all-gather."""

    @staticmethod
    def forward(ctx, x, group, axis):
        ctx.group, ctx.axis = group, axis
        n = _n(group)
        if n == 1:
            return x
        return x.chunk(n, dim=axis)[_r(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _gather(g, ctx.group, ctx.axis), None, None


class _Concat(torch.autograd.Function):
    """fwd: all-gather along last dim; bwd: keep this rank's slice."""

    @staticmethod
    def forward(ctx, x, group, axis):
        ctx.group, ctx.axis = group, axis
        return _gather(x, group, axis)

    @staticmethod
    def backward(ctx, g):
        n = _n(ctx.group)
        if n == 1:
            return g, None, None
        return g.chunk(n, dim=ctx.axis)[_r(ctx.group)].contiguous(), None, None


def _gather(x, group, axis):
    n = _n(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((n,) + tuple(x.shape), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=_pg(group))
    return torch.cat(list(out.unbind(0)), dim=axis)


def _static_value(x):
    """True while a static Program is being recorded and ``x`` is one of its (meta) values: the
    collective becomes ONE program node that runs the eager op (and its autograd) at replay, like the
    reference's c_identity / c_allreduce_sum / c_split / c_concat ops in a static program."""
    t = _unwrap(x) if isinstance(x, Tensor) else x
    if not isinstance(t, torch.Tensor) or not t.is_meta:
        return False
    from .....static.program import recording
    return recording()


def _record(eager, x, shape):
    from .....static.program import py_node, _paused
    t = _unwrap(x)
    with _paused():
        meta = torch.empty(shape, dtype=t.dtype, device='meta')
    return py_node(eager, [x], [meta])[0]


def _axis_shape(t, axis, f):
    shape = list(t.shape)
    shape[axis] = f(shape[axis])
    return shape


def _c_identity(x, group=None, skip_c_identity_dynamic=False):
    if _static_value(x):
        return _record(lambda v: _c_identity(v, group), x, list(_unwrap(x).shape))
    return _wrap(_Identity.apply(_unwrap(x), group))


def _mp_allreduce(x, op=None, group=None, use_calc_stream=True, use_model_parallel=True,
                  skip_c_identity_dynamic=False):
    if _static_value(x):
        return _record(lambda v: _mp_allreduce(v, group=group), x, list(_unwrap(x).shape))
    return _wrap(_AllReduce.apply(_unwrap(x), group))


def _c_split(x, group=None, axis=-1):
    if _static_value(x):
        n = _n(group)
        return _record(lambda v: _c_split(v, group, axis), x, _axis_shape(_unwrap(x), axis, lambda d: d // n))
    return _wrap(_Split.apply(_unwrap(x), group, axis))


def _c_concat(x, group=None, axis=-1):
    if _static_value(x):
        n = _n(group)
        return _record(lambda v: _c_concat(v, group, axis), x, _axis_shape(_unwrap(x), axis, lambda d: d * n))
    return _wrap(_Concat.apply(_unwrap(x), group, axis))


class _VocabParallelXent(torch.autograd.Function):
    """Softmax cross entropy over vocab-sharded logits [N, V/mp] (c_softmax_with_cross_entropy)."""

    @staticmethod
    def forward(ctx, logits, labels, group, ignore_index):
        n, r = _n(group), _r(group)
        x = logits.float()
        Vp = x.shape[-1]
        lo = r * Vp
        m = x.max(-1, keepdim=True)[0]
        if n > 1:
            dist.all_reduce(m, dist.ReduceOp.MAX, group=_pg(group))
        e = torch.exp(x - m)
        s = e.sum(-1, keepdim=True)
        local = (labels >= lo) & (labels < lo + Vp)
        idx = torch.where(local, labels - lo, torch.zeros_like(labels))
        tgt = torch.where(local, x.gather(-1, idx.unsqueeze(-1)).squeeze(-1), torch.zeros_like(m.squeeze(-1)))
        if n > 1:
            both = torch.stack([s.squeeze(-1), tgt], 0)
            dist.all_reduce(both, group=_pg(group))
            s, tgt = both[0].unsqueeze(-1), both[1]
        loss = (torch.log(s).squeeze(-1) + m.squeeze(-1) - tgt)
        valid = labels != ignore_index
        loss = torch.where(valid, loss, torch.zeros_like(loss))
        ctx.save_for_backward(e, s, idx, local, valid)
        ctx.dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        e, s, idx, local, valid = ctx.saved_tensors
        p = e / s
        oh = torch.zeros_like(p).scatter_(-1, idx.unsqueeze(-1), local.unsqueeze(-1).to(p.dtype))
        gr = (p - oh) * (g * valid.to(g.dtype)).unsqueeze(-1)
        return gr.to(ctx.dtype), None, None, None


def _c_softmax_with_cross_entropy(logits, label, group=None, return_softmax=False, ignore_index=-100):
    if _static_value(logits):
        from .....static.program import py_node, _paused
        t = _unwrap(logits)
        with _paused():
            meta = torch.empty(list(t.shape[:-1]) + [1], dtype=t.dtype, device='meta')
        return py_node(lambda lg, lb: _c_softmax_with_cross_entropy(lg, lb, group, False, ignore_index),
                       [logits, label], [meta])[0]
    lab = _unwrap(label)
    if lab.dim() == _unwrap(logits).dim():
        lab = lab.squeeze(-1)
    loss = _VocabParallelXent.apply(_unwrap(logits), lab.long(), group, ignore_index)
    return _wrap(loss.unsqueeze(-1))
