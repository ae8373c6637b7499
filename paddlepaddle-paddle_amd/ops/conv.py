"""NHWC conv2d forward on the hand-written implicit-GEMM MFMA kernel (csrc/conv.hip).

Reference: paddle/phi/kernels/gpudnn/conv_kernel.cu (forward), conv_grad_kernel.cu (backward).
Forward runs csrc/conv.hip (im2col folded into the LDS-DMA source addresses, zero padding via a
zero block, bias fused); the weight is packed into the [Cout][R][S][C]
k-contiguous image the kernel stages (re-packed per call).  Backward: the stride-1 data gradient is the same kernel
run on dY with the flipped, transposed filter; the 1x1 filter gradient is the hand-written GEMM
(dY^T X, split-K over pixels); strided data gradients and k>1 filter gradients use the storage
layer's convolution backward (MIOpen NHWC kernels).
"""
import os

import torch

from . import _native as N

_enabled = os.environ.get('PADDLE_AMD_HIP_CONV', '1') != '0'
_bwd_enabled = os.environ.get('PADDLE_AMD_HIP_CONV_BWD', '1') != '0'


def supported(x, w, groups):
    if not _enabled or groups != 1 or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if x.dim() != 4 or w.dim() != 4 or not x.is_cuda:
        return False
    if N.lib is None and N._load() is None:
        return False
    Cout, C, R, S = w.shape
    return x.shape[3] == C and bool(N.lib.pa_conv2d_fwd_ok(C, Cout, R, S))


def _packed(w):
    """[Cout][R][S][C] image of an OIHW filter.  Re-packed on every call: the fused optimizer
    kernels update parameters in place through raw pointers, which does not bump the tensor
    version counter, so no cache keyed on the tensor could tell a stale image (one small copy
    per conv per step)."""
    return w.detach().permute(0, 2, 3, 1).contiguous()


def _out_hw(H, W, R, S, stride, pad, dil):
    return ((H + 2 * pad[0] - dil[0] * (R - 1) - 1) // stride[0] + 1,
            (W + 2 * pad[1] - dil[1] * (S - 1) - 1) // stride[1] + 1)


def _fwd_packed(x, wpk, b, stride, pad, dil):
    """x: [N,H,W,C] bf16, wpk: packed [Cout][R][S][C] -> y [N,Ho,Wo,Cout]."""
    x = x.contiguous()
    Nb, H, W, C = x.shape
    Cout, R, S, _ = wpk.shape
    Ho, Wo = _out_hw(H, W, R, S, stride, pad, dil)
    y = torch.empty(Nb, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    bb = b.to(torch.bfloat16).contiguous() if b is not None else None
    N.check(N.lib.pa_conv2d_fwd(N.ptr(x), N.ptr(wpk), N.ptr(y), N.ptr(bb), Nb, H, W, C, Cout, R, S, stride[0],
                                stride[1], pad[0], pad[1], dil[0], dil[1], Ho, Wo, N.stream()), 'conv2d_fwd')
    return y


def conv2d_fwd(x, w, b, stride, pad, dil):
    """x: [N,H,W,C] bf16 (NHWC), w: [Cout,C,R,S] (paddle OIHW) -> y [N,Ho,Wo,Cout]."""
    return _fwd_packed(x, _packed(w), b, stride, pad, dil)


def _bwd_wins(dy, x):
    """Where the hand-written backward beat MIOpen's NHWC backward on MI355X (tools/conv_bench.py,
    ResNet50 shapes at batch 256): small spatial extents, or 28x28 maps with >= 256 input
    channels.  The 56x56 / narrow-channel layers stay on MIOpen."""
    pix = dy.shape[1] * dy.shape[2]
    return pix <= 196 or (pix <= 784 and x.shape[3] >= 256)


def _dgrad_ok(w, stride):
    Cout, C, R, S = w.shape
    return _bwd_enabled and tuple(stride) == (1, 1) and bool(N.lib.pa_conv2d_fwd_ok(Cout, C, R, S))


def conv2d_dgrad(dy, w, x_hw, pad, dil):
    """Stride-1 data gradient as a forward conv of dy with the spatially flipped, transposed
    filter ([C][R][S][Cout] image) and padding dil*(R-1) - pad (same kernel as the forward)."""
    Cout, C, R, S = w.shape
    wpk = w.detach().flip(2, 3).permute(1, 2, 3, 0).contiguous()
    p2 = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
    if p2[0] < 0 or p2[1] < 0:
        return None
    gx = _fwd_packed(dy, wpk, None, (1, 1), p2, dil)
    return gx if tuple(gx.shape[1:3]) == tuple(x_hw) else None


def conv2d_wgrad_1x1(dy, x):
    """1x1 / stride-1 / no-padding filter gradient: dW[co, c] = sum_pixels dY[p, co] X[p, c] on the
    hand-written GEMM (A = dY^T read with tr_b16; split-K over pixels when the output is small)."""
    from . import gemm
    Cout, C = dy.shape[-1], x.shape[-1]
    dy2, x2 = dy.reshape(-1, Cout), x.reshape(-1, C)
    a = dy2.t()
    tiles = -(-Cout // 256) * -(-C // 256)
    sk = 1
    while sk * 2 * tiles <= 256 and dy2.shape[0] % (64 * sk * 2) == 0:
        sk *= 2
    if not gemm.hip_mm_ok(a, x2, sk):
        return None
    return gemm.hip_mm(a, x2, splitk=sk).view(Cout, C, 1, 1)


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil):
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, dil, b is not None)
        return conv2d_fwd(x, w, b, stride, pad, dil)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, dil, has_b = ctx.cfg
        dy = dy.contiguous()
        gx = gw = gb = None
        dy_bwd_hip = _bwd_wins(dy, x)
        if ctx.needs_input_grad[0] and dy_bwd_hip and _dgrad_ok(w, stride):
            gx = conv2d_dgrad(dy, w, x.shape[1:3], pad, dil)
        if (ctx.needs_input_grad[1] and dy_bwd_hip and _bwd_enabled and w.shape[2] == w.shape[3] == 1
                and tuple(stride) == (1, 1) and tuple(pad) == (0, 0)):
            gw = conv2d_wgrad_1x1(dy, x)
            gw = gw.to(w.dtype) if gw is not None else None
        if has_b and ctx.needs_input_grad[2]:
            gb = dy.sum((0, 1, 2), dtype=torch.float32).to(dy.dtype)
        mask = [ctx.needs_input_grad[0] and gx is None, ctx.needs_input_grad[1] and gw is None, False]
        if any(mask):  # what the hand-written kernels do not cover: MIOpen NHWC backward
            lx, lw, _ = torch.ops.aten.convolution_backward(
                dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, None, list(stride), list(pad), list(dil), False,
                [0, 0], 1, mask)
            if mask[0]:
                gx = lx.permute(0, 2, 3, 1)
            if mask[1]:
                gw = lw
        return gx, gw, gb, None, None, None


def conv2d_nhwc(x, w, b, stride, pad, dil):
    return _Conv2dNHWC.apply(x, w, b, tuple(stride), tuple(pad), tuple(dil))
