"""LSQ+ fake quantisers with learned step sizes (and offset, for asymmetric activations).

Reference: python/paddle/nn/quant/lsq.py (LsqFunc:32, LsqPlusActFunc:101, FakeQuantActLSQPlus:138,
FakeQuantWeightLSQPlus:245).  Forward q = clip(round((x - beta) / s), Qn, Qp) * s + beta with
round-half-away-from-zero; backward: straight-through for x inside [Qn, Qp], the LSQ step-size
gradient  g * sum(dy * (Qn | Qp | round(q) - q))  for s and  g * sum(dy outside the range)  for beta,
g = 1 / sqrt(numel * Qp).  Initialisation over the first ``batch_init`` batches from the running
min/max (activations) or mean ± 3 std (weights), as the reference.
"""
import math

import torch

from ...core.tensor import _wrap, _unwrap
from ..layer.layers import Layer

__all__ = ['FakeQuantActLSQPlus', 'FakeQuantWeightLSQPlus']


def _round(x):
    return torch.sign(x) * torch.floor(x.abs() + 0.5)


class _Lsq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s, beta, g, Qn, Qp, axis):
        # s broadcasts against x (per-channel: shaped for the channel axis)
        q = (x - beta) / s
        ctx.save_for_backward(q)
        ctx.other = (g, Qn, Qp, axis, s.shape, beta is not None and beta.requires_grad)
        return torch.clamp(_round(q), Qn, Qp) * s + beta

    @staticmethod
    def backward(ctx, dy):
        q, = ctx.saved_tensors
        g, Qn, Qp, axis, sshape, want_beta = ctx.other
        lo, hi = (q < Qn).to(dy.dtype), (q > Qp).to(dy.dtype)
        mid = 1.0 - lo - hi
        ds_el = (lo * Qn + hi * Qp + mid * (_round(q) - q)) * dy * g
        if axis is None:
            ds = ds_el.sum().reshape(sshape)
        else:
            dims = [d for d in range(dy.dim()) if d != axis]
            ds = ds_el.sum(dim=dims).reshape(sshape)
        db = ((lo + hi) * dy * g).sum().reshape(()) if want_beta else None
        return mid * dy, ds, db, None, None, None, None


def _bounds(bits, all_positive):
    return (0, 2 ** bits - 1) if all_positive else (-(2 ** (bits - 1)), 2 ** (bits - 1) - 1)


class FakeQuantActLSQPlus(Layer):
    def __init__(self, quant_bits, all_positive=False, symmetric=False, batch_init=20, dtype='float32', name=None,
                 reduce_type=None):
        super().__init__()
        self.bits, self.all_positive, self.symmetric = quant_bits, all_positive, symmetric
        self.batch_init, self.name, self.reduce_type = batch_init, name, reduce_type
        self.Qn, self.Qp = _bounds(quant_bits, all_positive)
        from ..initializer import Constant
        self.s = self.create_parameter(shape=[], dtype='float32', default_initializer=Constant(1.0))
        self.s.stop_gradient = False
        self.beta = None
        if not symmetric:
            self.beta = self.create_parameter(shape=[], dtype='float32', default_initializer=Constant(0.0))
            self.beta.stop_gradient = False
        self.init_state = 0
        self.g = None

    def _sync(self):
        if self.reduce_type == 'max':
            import torch.distributed as dist
            if dist.is_initialized():
                with torch.no_grad():
                    dist.all_reduce(self.s._t, op=dist.ReduceOp.MAX)
                    if self.beta is not None:
                        dist.all_reduce(self.beta._t, op=dist.ReduceOp.MAX)

    def forward(self, activation):
        x = _unwrap(activation)
        self._sync()
        with torch.no_grad():
            lo, hi = x.detach().min().float(), x.detach().max().float()
            rng = (hi - lo) / (self.Qp - self.Qn)
            if self.init_state == 0:
                self.g = 1.0 / math.sqrt(x.numel() * self.Qp)
                self.s._t.copy_(rng)
                if self.beta is not None:
                    self.beta._t.copy_(lo - self.s._t * self.Qn)
            elif self.init_state < self.batch_init:
                self.s._t.copy_(self.s._t * 0.9 + 0.1 * rng)
                if self.beta is not None:
                    self.beta._t.copy_(self.beta._t * 0.9 + 0.1 * (lo - self.s._t * self.Qn))
        self.init_state += 1
        beta = self.beta._t if self.beta is not None else torch.zeros((), device=x.device)
        y = _Lsq.apply(x.float(), self.s._t, beta, self.g, self.Qn, self.Qp, None)
        return _wrap(y.to(x.dtype))


class FakeQuantWeightLSQPlus(Layer):
    def __init__(self, quant_bits, all_positive=False, per_channel=False, batch_init=20, channel_num=None,
                 quant_linear=False, dtype='float32', name=None, reduce_type=None):
        super().__init__()
        self.bits, self.all_positive, self.per_channel = quant_bits, all_positive, per_channel
        self.quant_linear, self.batch_init, self.name, self.reduce_type = quant_linear, batch_init, name, reduce_type
        self.quant_axis = 1 if quant_linear else 0
        self.collect_axis = 0 if quant_linear else 1
        self.Qn, self.Qp = _bounds(quant_bits, all_positive)
        from ..initializer import Constant
        self.s = self.create_parameter(shape=[channel_num or 1], dtype=dtype, default_initializer=Constant(1.0))
        self.s.stop_gradient = False
        self.init_state = 0
        self.g = None
        self.div = 2 ** quant_bits - 1

    def _stat(self, w):
        if self.per_channel:
            wt = w.reshape(w.shape[0], -1)
            mean, std = wt.mean(dim=self.collect_axis), wt.std(dim=self.collect_axis)
            return torch.maximum((mean - 3 * std).abs(), (mean + 3 * std).abs())
        mean, std = w.mean(), w.std()
        return torch.maximum((mean - 3 * std).abs(), (mean + 3 * std).abs()).reshape(1)

    def forward(self, weight):
        w = _unwrap(weight)
        if self.reduce_type == 'max':
            import torch.distributed as dist
            if dist.is_initialized():
                with torch.no_grad():
                    dist.all_reduce(self.s._t, op=dist.ReduceOp.MAX)
        with torch.no_grad():
            st = self._stat(w.detach().float()).to(self.s._t.dtype)
            if self.init_state == 0:
                self.g = 1.0 / math.sqrt(w.numel() * self.Qp)
                self.s._t.copy_((st / self.div).expand_as(self.s._t))
            elif self.init_state < self.batch_init:
                self.s._t.copy_(self.s._t * 0.9 + 0.1 * st / self.div)
        self.init_state += 1
        if self.per_channel:
            shape = [1] * w.dim()
            shape[self.quant_axis] = -1
            s = self.s._t.reshape(shape)
            axis = self.quant_axis
        else:
            s = self.s._t.reshape([1] * w.dim()) if w.dim() else self.s._t.reshape(())
            axis = None
        y = _Lsq.apply(w.float(), s, torch.zeros((), device=w.device), self.g, self.Qn, self.Qp, axis)
        return _wrap(y.to(w.dtype))
