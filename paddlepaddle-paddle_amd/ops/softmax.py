"""Row softmax (+ causal upper-triangle mask) on csrc/softmax_xent.hip.

Reference: paddle/phi/kernels/gpudnn/softmax_gpudnn.h,
paddle/phi/kernels/fusion/gpu/fused_softmax_mask_upper_triangle_kernel.cu.
"""
import torch

from . import _native as N


class _Softmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, causal_S):
        cols = x.shape[-1]
        x2 = x.contiguous()
        rows = x2.numel() // cols
        y = torch.empty_like(x2)
        N.check(N.lib.pa_softmax_fwd(N.ptr(x2), N.ptr(y), rows, cols, causal_S, N.dtcode(x.dtype), N.stream()),
                'softmax_fwd')
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, = ctx.saved_tensors
        cols = y.shape[-1]
        rows = y.numel() // cols
        dy = dy.contiguous()
        dx = torch.empty_like(y)
        N.check(N.lib.pa_softmax_bwd(N.ptr(y), N.ptr(dy), N.ptr(dx), rows, cols, N.dtcode(y.dtype), N.stream()),
                'softmax_bwd')
        return dx, None


def softmax(x):
    return _Softmax.apply(x, 0)


def softmax_mask_upper_triangle(x):
    """softmax over the last dim of [..., S, S] scores with keys > query masked (fused causal)."""
    return _Softmax.apply(x, x.shape[-2])
