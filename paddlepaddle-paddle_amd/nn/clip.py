"""Gradient clipping (reference: python/paddle/nn/clip.py).

ClipGradByGlobalNorm computes the global norm with ONE fused multi-tensor reduction
(torch._foreach_norm → per-tensor norms → one stack/norm) and scales in place with
_foreach_mul_, so clipping costs two launches regardless of the parameter count.
"""
import torch

from ..core.tensor import Tensor, _wrap, _unwrap


class ClipGradBase:
    def __call__(self, params_grads):
        return self._dygraph_clip(params_grads)


class ClipGradByValue(ClipGradBase):
    def __init__(self, max, min=None):  # noqa: A002
        self.max = float(max)
        self.min = -self.max if min is None else float(min)

    def _dygraph_clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is not None and getattr(p, 'need_clip', True):
                g._t.clamp_(self.min, self.max)
            out.append((p, g))
        return out


class ClipGradByNorm(ClipGradBase):
    def __init__(self, clip_norm):
        self.clip_norm = float(clip_norm)

    def _dygraph_clip(self, params_grads):
        out = []
        for p, g in params_grads:
            if g is not None and getattr(p, 'need_clip', True):
                n = g._t.float().norm()
                g._t.mul_(torch.clamp(self.clip_norm / torch.clamp(n, min=self.clip_norm), max=1.0).to(g._t.dtype))
            out.append((p, g))
        return out


class ClipGradByGlobalNorm(ClipGradBase):
    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = float(clip_norm)
        self.group_name = group_name
        self._extra_sq_norm_fn = None  # hook used by distributed wrappers (sharding / TP) to all-reduce

    def global_norm(self, grads):
        if not grads:
            return None
        norms = torch._foreach_norm([g.float() if g.dtype != torch.float32 else g for g in grads])
        sq = torch.stack(norms).square().sum()
        if self._extra_sq_norm_fn is not None:
            sq = self._extra_sq_norm_fn(sq)
        return sq.sqrt()

    def _dygraph_clip(self, params_grads):
        grads = [g._t for p, g in params_grads if g is not None and getattr(p, 'need_clip', True)]
        if not grads:
            return params_grads
        gn = self.global_norm(grads)
        scale = torch.clamp(self.clip_norm / torch.clamp(gn, min=self.clip_norm), max=1.0)
        by_dtype = {}
        for g in grads:
            by_dtype.setdefault(g.dtype, []).append(g)
        for dt, gs in by_dtype.items():
            torch._foreach_mul_(gs, scale.to(dt))
        return params_grads


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    ps = [parameters] if isinstance(parameters, Tensor) else list(parameters)
    grads = [p._t.grad for p in ps if p._t.grad is not None]
    if not grads:
        return _wrap(torch.tensor(0.0))
    total = torch.nn.utils.clip_grad_norm_([p._t for p in ps], max_norm, norm_type, error_if_nonfinite)
    return _wrap(total)


def clip_grad_value_(parameters, clip_value):
    ps = [parameters] if isinstance(parameters, Tensor) else list(parameters)
    torch.nn.utils.clip_grad_value_([p._t for p in ps], clip_value)
