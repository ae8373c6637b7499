"""LayerNorm / RMSNorm (+ fused residual add) on csrc/norm.hip.

Reference: paddle/phi/kernels/gpu/layer_norm_kernel.cu, incubate fused_rms_norm /
fused_layer_norm (residual variant returns the pre-norm sum as the new residual stream).
"""
import torch

from . import _native as N


def _live(t, what):
    if t is not None and t.untyped_storage().nbytes() == 0:
        raise RuntimeError(f"{what} storage is released (a sharding stage-3 unit used outside its layer's forward?)")


def _fwd(x, res, w, b, eps, rms):
    _live(w, 'norm weight')
    _live(b, 'norm bias')
    cols = x.shape[-1]
    x2 = x.contiguous()
    rows = x2.numel() // cols
    y = torch.empty_like(x2)
    s = torch.empty_like(x2) if res is not None else None
    r2 = res.contiguous() if res is not None else None
    rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
    xd, wd = N.dtcode(x.dtype), N.dtcode(w.dtype)
    if rms:
        N.check(N.lib.pa_rmsnorm_fwd(N.ptr(x2), N.ptr(r2), N.ptr(w), N.ptr(y), N.ptr(s), N.ptr(rstd), rows, cols, eps,
                                     xd, wd, N.stream()), 'rmsnorm_fwd')
        mean = None
    else:
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        N.check(N.lib.pa_layernorm_fwd(N.ptr(x2), N.ptr(r2), N.ptr(w), N.ptr(b), N.ptr(y), N.ptr(s), N.ptr(mean),
                                       N.ptr(rstd), rows, cols, eps, xd, wd, N.stream()), 'layernorm_fwd')
    return y, s, mean, rstd


def _bwd(dy, xin, w, mean, rstd, dsum, rms, need_b):
    cols = xin.shape[-1]
    rows = xin.numel() // cols
    dy = dy.contiguous()
    dx = torch.empty_like(xin)
    np_ = N.lib.pa_norm_bwd_nparts(rows)
    part = torch.empty(2 * np_ * cols, dtype=torch.float32, device=xin.device)
    dw = torch.empty_like(w)
    xd, wd = N.dtcode(xin.dtype), N.dtcode(w.dtype)
    ds = dsum.contiguous() if dsum is not None else None
    if rms:
        N.check(N.lib.pa_rmsnorm_bwd(N.ptr(dy), N.ptr(xin), N.ptr(w), N.ptr(rstd), N.ptr(ds), N.ptr(dx), N.ptr(part),
                                     N.ptr(dw), rows, cols, xd, wd, N.stream()), 'rmsnorm_bwd')
        return dx, dw, None
    db = torch.empty_like(w) if need_b else None
    N.check(N.lib.pa_layernorm_bwd(N.ptr(dy), N.ptr(xin), N.ptr(w), N.ptr(mean), N.ptr(rstd), N.ptr(ds), N.ptr(dx),
                                   N.ptr(part), N.ptr(dw), N.ptr(db), rows, cols, xd, wd, N.stream()), 'layernorm_bwd')
    return dx, dw, db


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        y, _, mean, rstd = _fwd(x, None, w, b, eps, False)
        ctx.save_for_backward(x, w, mean, rstd)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, mean, rstd = ctx.saved_tensors
        dx, dw, db = _bwd(dy, x.contiguous(), w, mean, rstd, None, False, ctx.has_b)
        return dx, dw, db, None


class _RMSNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, eps):
        y, _, _, rstd = _fwd(x, None, w, None, eps, True)
        ctx.save_for_backward(x, w, rstd)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, rstd = ctx.saved_tensors
        dx, dw, _ = _bwd(dy, x.contiguous(), w, None, rstd, None, True, False)
        return dx, dw, None


class _AddNorm(torch.autograd.Function):
    """(y, s) = (norm(x + r), x + r): one pass reads x, r and writes y, s."""

    @staticmethod
    def forward(ctx, x, r, w, b, eps, rms):
        y, s, mean, rstd = _fwd(x, r, w, b, eps, rms)
        ctx.save_for_backward(s, w, mean, rstd)
        ctx.rms, ctx.has_b = rms, b is not None
        ctx.set_materialize_grads(False)  # an unused sum output (post-LN blocks) costs no zero tensor
        return y, s

    @staticmethod
    def backward(ctx, dy, ds):
        s, w, mean, rstd = ctx.saved_tensors
        if dy is None:
            dy = torch.zeros_like(s)
        dx, dw, db = _bwd(dy, s, w, mean, rstd, ds, ctx.rms, ctx.has_b)
        return dx, dx, dw, db, None, None


def layer_norm(x, w, b, eps):
    return _LayerNorm.apply(x, w, b, eps)


def rms_norm(x, w, eps):
    return _RMSNorm.apply(x, w, eps)


def add_layer_norm(x, residual, w, b, eps):
    return _AddNorm.apply(x, residual, w, b, eps, False)


def add_rms_norm(x, residual, w, eps):
    return _AddNorm.apply(x, residual, w, None, eps, True)
