"""Fused activation / dropout ops on csrc/act.hip.

Reference: paddle/phi/kernels/fusion/gpu/fused_bias_act_kernel.cu, fused_dropout_add_kernel.cu,
incubate swiglu.  Dropout keep-masks are regenerated from (seed, offset) in backward.
"""
import torch

from . import _native as N

GELU, GELU_TANH, SILU, RELU, IDENT = 0, 1, 2, 3, 4


def _vec_ok(t, cols):
    e = 16 // t.element_size()
    return cols % e == 0


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act):
        x2 = x.contiguous()
        cols = x2.shape[-1]
        y = torch.empty_like(x2)
        N.check(N.lib.pa_bias_act(act, 0, None, N.ptr(x2), N.ptr(bias), N.ptr(y), x2.numel(), cols,
                                  N.dtcode(x.dtype), N.stream()), 'bias_act_fwd')
        ctx.save_for_backward(x2, bias)
        ctx.act = act
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bias = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        N.check(N.lib.pa_bias_act(ctx.act, 1, N.ptr(dy), N.ptr(x), N.ptr(bias), N.ptr(dx), x.numel(), x.shape[-1],
                                  N.dtcode(x.dtype), N.stream()), 'bias_act_bwd')
        db = dx.reshape(-1, x.shape[-1]).sum(0, dtype=torch.float32).to(bias.dtype) if bias is not None else None
        return dx, db, None


def _apply(x, bias, act, torch_fn):
    cols = x.shape[-1]
    if not _vec_ok(x, cols) or (bias is not None and bias.dtype != x.dtype):
        return torch_fn(x if bias is None else x + bias)
    return _BiasAct.apply(x, bias, act)


def gelu(x, approximate=False, bias=None):
    tf = lambda v: torch.nn.functional.gelu(v, approximate='tanh' if approximate else 'none')  # noqa: E731
    return _apply(x, bias, GELU_TANH if approximate else GELU, tf)


def silu(x, bias=None):
    return _apply(x, bias, SILU, torch.nn.functional.silu)


def bias_relu(x, bias=None):
    return _apply(x, bias, RELU, torch.relu)


class _Swiglu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        cols = a.shape[-1]
        rows = a.numel() // cols
        y = torch.empty(*a.shape, dtype=a.dtype, device=a.device)
        N.check(N.lib.pa_swiglu_fwd(N.ptr(a), N.ptr(b), N.ptr(y), rows * cols, a.stride(-2) if a.dim() > 1 else cols,
                                    cols, N.dtcode(a.dtype), N.stream()), 'swiglu_fwd')
        ctx.save_for_backward(a, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        a, b = ctx.saved_tensors
        cols = a.shape[-1]
        rows = a.numel() // cols
        stride = a.stride(-2) if a.dim() > 1 else cols
        dy = dy.contiguous()
        if a.is_contiguous() and b.is_contiguous():
            da, db = torch.empty_like(a), torch.empty_like(b)
            st = cols
        else:  # a, b are halves of one [rows, 2*cols] buffer: write grads into one buffer too
            buf = torch.empty(rows, stride, dtype=a.dtype, device=a.device)
            da, db = buf[:, :cols], buf[:, cols:2 * cols]
            st = stride
        N.check(N.lib.pa_swiglu_bwd(N.ptr(a), N.ptr(b), N.ptr(dy), N.ptr(da), N.ptr(db), rows * cols, st, cols,
                                    N.dtcode(a.dtype), N.stream()), 'swiglu_bwd')
        return da.reshape(a.shape), db.reshape(b.shape)


class _SwigluPacked(torch.autograd.Function):
    """silu(x[..., :C]) * x[..., C:] of one [rows, 2C] tensor (the fused gate/up projection):
    the gradient is ONE [rows, 2C] buffer written by the backward kernel, so autograd never
    concatenates per-half gradients (the chunk() backward copied the whole 2C-wide gradient)."""

    @staticmethod
    def forward(ctx, x):
        cols = x.shape[-1] // 2
        x2 = x.reshape(-1, 2 * cols)
        rows = x2.shape[0]
        y = torch.empty(rows, cols, dtype=x.dtype, device=x.device)
        N.check(N.lib.pa_swiglu_fwd(N.ptr(x2), N.ptr(x2[:, cols:]), N.ptr(y), rows * cols, 2 * cols, cols,
                                    N.dtcode(x.dtype), N.stream()), 'swiglu_fwd')
        ctx.save_for_backward(x2)
        ctx.xshape = x.shape
        return y.reshape(*x.shape[:-1], cols)

    @staticmethod
    def backward(ctx, dy):
        x2, = ctx.saved_tensors
        rows, cols = x2.shape[0], x2.shape[1] // 2
        dy = dy.contiguous()
        dx = torch.empty_like(x2)
        N.check(N.lib.pa_swiglu_bwd(N.ptr(x2), N.ptr(x2[:, cols:]), N.ptr(dy), N.ptr(dx), N.ptr(dx[:, cols:]),
                                    rows * cols, 2 * cols, cols, N.dtcode(x2.dtype), N.stream()), 'swiglu_bwd')
        return dx.reshape(ctx.xshape)


def swiglu_packed_ok(x):
    cols = x.shape[-1] // 2 if x.dim() >= 1 else 0
    return (x.is_cuda and x.is_contiguous() and x.shape[-1] % 2 == 0 and x.dtype in (torch.bfloat16, torch.float16)
            and _vec_ok(x[..., :cols], cols))


def swiglu_packed(x):
    return _SwigluPacked.apply(x)


def swiglu(a, b):
    cols = a.shape[-1]
    ok = (_vec_ok(a, cols) and a.stride(-1) == 1 and b.stride(-1) == 1 and a.stride() == b.stride()
          and (a.is_contiguous() or (a.dim() >= 2 and a.reshape(-1, cols).stride(0) == a.stride(-2))))
    if not ok:
        return torch.nn.functional.silu(a) * b
    if a.dim() > 2:
        a2 = a.reshape(-1, cols) if a.is_contiguous() else a.flatten(0, -2)
        b2 = b.reshape(-1, cols) if b.is_contiguous() else b.flatten(0, -2)
        return _Swiglu.apply(a2, b2).reshape(*a.shape)
    return _Swiglu.apply(a, b)


def _next_seed(n):
    """(seed, offset) from the paddle.seed-controlled host generator (see ops.fused._next_seed)."""
    from ..device.cuda.graphs import host_rng_guard
    host_rng_guard('dropout_add')
    seed, off = torch.randint(0, 2 ** 31 - 1, (2,), device='cpu').tolist()
    return seed, off


class _DropoutAdd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, residual, p):
        x2 = x.contiguous()
        r2 = residual.contiguous() if residual is not None else None
        y = torch.empty_like(x2)
        seed, off = _next_seed(x2.numel())
        N.check(N.lib.pa_dropout_add_fwd(N.ptr(x2), N.ptr(r2), N.ptr(y), x2.numel(), p, seed, off,
                                         N.dtcode(x.dtype), N.stream()), 'dropout_add_fwd')
        ctx.seed, ctx.off, ctx.p = seed, off, p
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        N.check(N.lib.pa_dropout_bwd(N.ptr(dy), N.ptr(dx), dy.numel(), ctx.p, ctx.seed, ctx.off, N.dtcode(dy.dtype),
                                     N.stream()), 'dropout_bwd')
        return dx, (dy if ctx.has_res else None), None


def dropout(x, p):
    return _DropoutAdd.apply(x, None, p)


def dropout_add(x, residual, p):
    """residual + dropout(x, p) in one pass (paddle.incubate.nn.functional.fused_dropout_add)."""
    if p == 0.0:
        return x + residual
    return _DropoutAdd.apply(x, residual, p)
