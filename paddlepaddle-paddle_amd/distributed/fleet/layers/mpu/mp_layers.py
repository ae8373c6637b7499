"""Tensor-parallel layers (reference: python/paddle/distributed/fleet/layers/mpu/mp_layers.py:
VocabParallelEmbedding:47, ColumnParallelLinear:334, RowParallelLinear:541, ParallelCrossEntropy:742).

Weights are the local shard (paddle layout [in, out/mp] for column, [in/mp, out] for row),
created on every rank from the model-parallel RNG stream so shards differ across ranks and
agree with a single-device model initialised from the same full weight.
"""
import torch

from .....nn.layer.layers import Layer
from .....nn import functional as F
from .....nn import initializer as I
from .....core.tensor import Tensor, _wrap, _unwrap
from . import mp_ops


def _hcg_group():
    from ... import _inited, get_hybrid_communicate_group
    hcg = get_hybrid_communicate_group() if _inited() else None
    return hcg.get_model_parallel_group() if hcg is not None else None


def _size_rank(group):
    return mp_ops._n(group), mp_ops._r(group)


def _mp_async_allreduce():
    """strategy.hybrid_configs['mp_configs']['mp_async_allreduce'] (default True here)."""
    from ... import fleet as _fleet
    st = getattr(_fleet, '_strategy', None)
    cfg = (getattr(st, 'hybrid_configs', None) or {}).get('mp_configs', {}) if st is not None else {}
    return bool(cfg.get('mp_async_allreduce', True))


class _ColumnParallelLinearFn(torch.autograd.Function):
    """Column-parallel Linear with the input-gradient all-reduce overlapped with the weight-gradient
    GEMM (reference: distributed/passes/allreduce_matmul_grad_overlapping.py:37 and the
    mp_async_allreduce path of mp_layers.py).  Backward: dX = dY W^T, launch its all-reduce over the
    mp group asynchronously (RCCL on its own stream), compute dW = X^T dY and db while it runs, wait.
    Under a zero-bubble pipeline (WeightGradStore active) dW / db are queued for the W pass instead."""

    @staticmethod
    def forward(ctx, x, w, b, wp, bp, group):
        ctx.save_for_backward(x, w)
        ctx.wp, ctx.bp, ctx.group = wp, bp, group
        from .....ops import matmul as _mm
        return _mm.linear(x, w, b)

    @staticmethod
    def backward(ctx, dy):
        import torch.distributed as dist
        x, w = ctx.saved_tensors
        dx = torch.matmul(dy, w.t()).contiguous()
        work = dist.all_reduce(dx, group=mp_ops._pg(ctx.group), async_op=True)
        need_w = ctx.needs_input_grad[1]
        need_b = ctx.needs_input_grad[2]
        dw = db = None
        if need_w or need_b:
            x2 = x.reshape(-1, x.shape[-1])
            dy2 = dy.reshape(-1, dy.shape[-1])
            from ...meta_parallel.zero_bubble_utils import WeightGradStore, _accumulate
            if WeightGradStore.active:
                from .....parallel.flat_buffer import defer_grad
                wp, bp = ctx.wp, ctx.bp
                if need_w:
                    defer_grad(wp)
                if need_b:
                    defer_grad(bp)
                x2d, dy2d = x2.detach(), dy2.detach()

                def w_pass():
                    if need_w:
                        _accumulate(wp, x2d.t().matmul(dy2d))
                    if need_b:
                        _accumulate(bp, dy2d.sum(0))
                WeightGradStore.put(w_pass)
            else:
                dw = x2.t().matmul(dy2) if need_w else None  # overlaps the all-reduce of dx
                db = dy2.sum(0) if need_b else None
        work.wait()
        return dx, dw, db, None, None, None


class VocabParallelEmbedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, weight_attr=None, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _hcg_group()
        self.world_size, self.rank = _size_rank(self.model_parallel_group)
        self.origin_num_embeddings = num_embeddings
        self.is_mp = self.world_size > 1
        per = (num_embeddings + self.world_size - 1) // self.world_size
        self.vocab_start_index = self.rank * per
        self.vocab_end_index = min(num_embeddings, self.vocab_start_index + per)
        self.weight = self.create_parameter([per, embedding_dim], attr=weight_attr,
                                            default_initializer=I.XavierNormal())
        self.weight.is_distributed = self.is_mp
        self.weight.split_axis = 0

    def forward(self, x):
        ids = _unwrap(x)
        if not self.is_mp:
            return F.embedding(x, self.weight)
        lo, hi = self.vocab_start_index, self.vocab_end_index
        mask = (ids < lo) | (ids >= hi)
        local = torch.where(mask, torch.zeros_like(ids), ids - lo)
        out = _unwrap(F.embedding(_wrap(local), self.weight))
        out = out.masked_fill(mask.unsqueeze(-1), 0)
        return mp_ops._mp_allreduce(_wrap(out), group=self.model_parallel_group)


class ColumnParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=None, gather_output=True,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _hcg_group()
        self.world_size, self.rank = _size_rank(self.model_parallel_group)
        self.is_mp = self.world_size > 1
        assert out_features % self.world_size == 0, "out_features must be divisible by mp degree"
        self.output_size_per_partition = out_features // self.world_size
        self.gather_output = gather_output
        self.weight = self.create_parameter([in_features, self.output_size_per_partition], attr=weight_attr)
        self.weight.is_distributed = self.is_mp
        self.weight.split_axis = 1
        if has_bias is None or has_bias:
            self.bias = self.create_parameter([self.output_size_per_partition], is_bias=True)
            self.bias.is_distributed = self.is_mp
            self.bias.split_axis = 0
        else:
            self.bias = None

    def forward(self, x):
        from .....framework import in_dynamic_mode
        if self.is_mp and in_dynamic_mode() and torch.is_grad_enabled() and _mp_async_allreduce() and \
                not self.weight.stop_gradient:
            xt = _unwrap(x)
            w = self.weight._t
            b = self.bias._t if self.bias is not None else None
            if w.dtype != xt.dtype:  # AMP: compute in the activation dtype
                w = w.to(xt.dtype)
                b = b.to(xt.dtype) if b is not None else None
            out = _wrap(_ColumnParallelLinearFn.apply(xt, w, b, self.weight, self.bias, self.model_parallel_group))
            if self.gather_output:
                out = mp_ops._c_concat(out, group=self.model_parallel_group)
            return out
        if self.is_mp:
            x = mp_ops._c_identity(x, group=self.model_parallel_group)
        out = F.linear(x, self.weight, self.bias)
        if self.gather_output and self.is_mp:
            out = mp_ops._c_concat(out, group=self.model_parallel_group)
        return out


class RowParallelLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, has_bias=True, input_is_parallel=False,
                 fuse_matmul_bias=False, mp_group=None, name=None):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _hcg_group()
        self.world_size, self.rank = _size_rank(self.model_parallel_group)
        self.is_mp = self.world_size > 1
        assert in_features % self.world_size == 0, "in_features must be divisible by mp degree"
        self.input_size_per_partition = in_features // self.world_size
        self.input_is_parallel = input_is_parallel
        self.weight = self.create_parameter([self.input_size_per_partition, out_features], attr=weight_attr)
        self.weight.is_distributed = self.is_mp
        self.weight.split_axis = 0
        self.bias = self.create_parameter([out_features], is_bias=True) if has_bias else None

    def forward(self, x):
        if self.is_mp and not self.input_is_parallel:
            x = mp_ops._c_split(x, group=self.model_parallel_group)
        out = F.linear(x, self.weight, None)
        if self.is_mp:
            out = mp_ops._mp_allreduce(out, group=self.model_parallel_group)
        if self.bias is not None:
            out = out + self.bias
        return out


class ParallelCrossEntropy(Layer):
    def __init__(self, mp_group=None, name=None, ignore_index=-100):
        super().__init__()
        self.model_parallel_group = mp_group if mp_group is not None else _hcg_group()
        self.world_size, self.rank = _size_rank(self.model_parallel_group)
        self.ignore_index = ignore_index

    def forward(self, input, label):  # noqa: A002
        return mp_ops._c_softmax_with_cross_entropy(input, label, group=self.model_parallel_group,
                                                    ignore_index=self.ignore_index)
