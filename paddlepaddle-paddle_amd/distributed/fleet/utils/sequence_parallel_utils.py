"""Sequence parallelism (reference: python/paddle/distributed/fleet/utils/sequence_parallel_utils.py).

Activations outside the tensor-parallel regions are sharded along the SEQUENCE dim across the
mp group: LayerNorm/dropout run on S/mp tokens; entering a column-parallel linear all-gathers
the sequence (backward: reduce-scatter), leaving a row-parallel linear reduce-scatters it
(backward: all-gather) — replacing TP's all-reduce with RS+AG of the same bytes while cutting
activation memory by mp.  Layout: [S, B, H] (sequence-major, as the reference).
"""
import torch
import torch.distributed as dist

from ....core.tensor import Tensor, _wrap, _unwrap
from ....nn.layer.layers import Layer
from ....nn import functional as F
from ..layers.mpu.mp_layers import ColumnParallelLinear, RowParallelLinear, _hcg_group
from ..layers.mpu import mp_ops


def _grp(group):
    return group if group is not None else _hcg_group()


def _ag_seq(x, group):
    n = mp_ops._n(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((n * x.shape[0],) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=mp_ops._pg(group))
    return out


def _rs_seq(x, group):
    n = mp_ops._n(group)
    if n == 1:
        return x
    x = x.contiguous()
    out = torch.empty((x.shape[0] // n,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x, group=mp_ops._pg(group))
    return out


class _Scatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        n = mp_ops._n(group)
        return x if n == 1 else x.chunk(n, 0)[mp_ops._r(group)].contiguous()

    @staticmethod
    def backward(ctx, g):
        return _ag_seq(g, ctx.group), None


class _Gather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _ag_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        n = mp_ops._n(ctx.group)
        return (g if n == 1 else g.chunk(n, 0)[mp_ops._r(ctx.group)].contiguous()), None


class _AllGather(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _ag_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _rs_seq(g, ctx.group), None


class _ReduceScatter(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _rs_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _ag_seq(g, ctx.group), None


class ScatterOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_Scatter.apply(_unwrap(x), _grp(group)))


class GatherOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_Gather.apply(_unwrap(x), _grp(group)))


class AllGatherOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_AllGather.apply(_unwrap(x), _grp(group)))


class ReduceScatterOp:
    @staticmethod
    def apply(x, group=None):
        return _wrap(_ReduceScatter.apply(_unwrap(x), _grp(group)))


def mark_as_sequence_parallel_parameter(parameter):
    parameter.sequence_parallel = True


def is_sequence_parallel_parameter(parameter):
    return getattr(parameter, 'sequence_parallel', False)


def register_sequence_parallel_allreduce_hooks(model, accumulation_steps=1, fuse_sequence_parallel_allreduce=False):
    """Params replicated across mp but fed sequence-sharded activations (LayerNorm weights) need
    their gradients all-reduced over the mp group."""
    group = _hcg_group()
    if mp_ops._n(group) == 1:
        return
    params = [p for p in model.parameters() if is_sequence_parallel_parameter(p)]
    for p in params:
        p._t.register_post_accumulate_grad_hook(lambda t: dist.all_reduce(t.grad, group=mp_ops._pg(group)))


class ColumnSequenceParallelLinear(ColumnParallelLinear):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None, gather_output=False,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__(in_features, out_features, weight_attr, has_bias, False, fuse_matmul_bias, mp_group, name)

    def forward(self, x):
        full = AllGatherOp.apply(x, self.model_parallel_group) if self.is_mp else x
        return F.linear(full, self.weight, self.bias)


class RowSequenceParallelLinear(RowParallelLinear):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True, input_is_parallel=True,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__(in_features, out_features, weight_attr, has_bias, True, fuse_matmul_bias, mp_group, name)
        if self.bias is not None:
            mark_as_sequence_parallel_parameter(self.bias)

    def forward(self, x):
        out = F.linear(x, self.weight, None)
        if self.is_mp:
            out = ReduceScatterOp.apply(out, self.model_parallel_group)
        if self.bias is not None:
            out = out + self.bias
        return out
