"""NHWC conv2d forward on the hand-written implicit-GEMM MFMA kernel (csrc/conv.hip).

Reference: paddle/phi/kernels/gpudnn/conv_kernel.cu (forward), conv_grad_kernel.cu (backward).
Forward runs csrc/conv.hip (im2col folded into the LDS-DMA source addresses, zero padding via a
zero block, bias fused); the weight is packed once per weight version into the [Cout][R][S][C]
k-contiguous image the kernel stages.  Backward (data and filter gradients) uses the storage
layer's convolution backward (MIOpen NHWC kernels).
"""
import os

import torch

from . import _native as N

_enabled = os.environ.get('PADDLE_AMD_HIP_CONV', '1') != '0'
_pack_cache = {}


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
    key = id(w)
    ent = _pack_cache.get(key)
    ver = (w._version, w.data_ptr())
    if ent is None or ent[0] != ver:
        ent = (ver, w.detach().permute(0, 2, 3, 1).contiguous())
        _pack_cache[key] = ent
        if len(_pack_cache) > 512:
            _pack_cache.pop(next(iter(_pack_cache)))
    return ent[1]


def _out_hw(H, W, R, S, stride, pad, dil):
    return ((H + 2 * pad[0] - dil[0] * (R - 1) - 1) // stride[0] + 1,
            (W + 2 * pad[1] - dil[1] * (S - 1) - 1) // stride[1] + 1)


def conv2d_fwd(x, w, b, stride, pad, dil):
    """x: [N,H,W,C] bf16 (NHWC), w: [Cout,C,R,S] (paddle OIHW) -> y [N,Ho,Wo,Cout]."""
    x = x.contiguous()
    Nb, H, W, C = x.shape
    Cout, _, R, S = w.shape
    Ho, Wo = _out_hw(H, W, R, S, stride, pad, dil)
    y = torch.empty(Nb, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    bb = b.to(torch.bfloat16).contiguous() if b is not None else None
    N.check(N.lib.pa_conv2d_fwd(N.ptr(x), N.ptr(_packed(w)), N.ptr(y), N.ptr(bb), Nb, H, W, C, Cout, R, S, stride[0],
                                stride[1], pad[0], pad[1], dil[0], dil[1], Ho, Wo, N.stream()), 'conv2d_fwd')
    return y


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
        mask = [ctx.needs_input_grad[0], ctx.needs_input_grad[1], has_b and ctx.needs_input_grad[2]]
        gx, gw, gb = torch.ops.aten.convolution_backward(
            dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, [w.shape[0]] if has_b else None, list(stride),
            list(pad), list(dil), False, [0, 0], 1, mask)
        gx = gx.permute(0, 2, 3, 1) if gx is not None else None
        return gx, gw, gb, None, None, None


def conv2d_nhwc(x, w, b, stride, pad, dil):
    return _Conv2dNHWC.apply(x, w, b, tuple(stride), tuple(pad), tuple(dil))
