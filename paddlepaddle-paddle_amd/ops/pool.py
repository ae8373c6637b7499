"""Channels-last 2-D max pooling on csrc/pool.hip (one-byte argmax, gather backward).

Reference: paddle/phi/kernels/funcs/pooling.cu (MaxPool2dWithIndex*), used by
paddle.nn.functional.max_pool2d(data_format='NHWC').
"""
import torch

from . import _native as N


def _out_size(n, k, s, p, ceil_mode):
    num = n + 2 * p - k
    o = (-(-num // s) if ceil_mode else num // s) + 1
    if ceil_mode and (o - 1) * s >= n + p:  # last window must start inside the input (torch/paddle rule)
        o -= 1
    return o


def supported(x, k, s, p):
    """x: NHWC tensor on the GPU; k/s/p: 2-tuples."""
    if x.dim() != 4 or x.dtype not in (torch.bfloat16, torch.float16, torch.float32) or not x.is_cuda:
        return False
    e = 16 // x.element_size()
    return x.shape[3] % e == 0 and k[0] * k[1] <= 256 and all(0 <= p[i] < k[i] for i in range(2)) and \
        min(s) > 0 and N._load() is not None


class _MaxPoolNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, ceil_mode):
        x = x.contiguous()
        n, h, w, c = x.shape
        oh, ow = _out_size(h, k[0], s[0], p[0], ceil_mode), _out_size(w, k[1], s[1], p[1], ceil_mode)
        y = torch.empty((n, oh, ow, c), dtype=x.dtype, device=x.device)
        idx = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device)
        N.check(N.lib.pa_maxpool2d_nhwc_fwd(N.ptr(x), N.ptr(y), N.ptr(idx), n, h, w, c, oh, ow, k[0], k[1], s[0], s[1],
                                            p[0], p[1], N.dtcode(x.dtype), N.stream()), 'maxpool2d_nhwc_fwd')
        ctx.save_for_backward(idx)
        ctx.geo = (n, h, w, c, oh, ow, k, s, p)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        n, h, w, c, oh, ow, k, s, p = ctx.geo
        dy = dy.contiguous()
        dx = torch.empty((n, h, w, c), dtype=dy.dtype, device=dy.device)
        N.check(N.lib.pa_maxpool2d_nhwc_bwd(N.ptr(dy), N.ptr(idx), N.ptr(dx), n, h, w, c, oh, ow, k[0], k[1], s[0],
                                            s[1], p[0], p[1], N.dtcode(dy.dtype), N.stream()), 'maxpool2d_nhwc_bwd')
        return dx, None, None, None, None


def max_pool2d_nhwc(x, k, s, p, ceil_mode=False):
    if N._load() is None:
        raise RuntimeError("max_pool2d_nhwc: HIP kernel library not loaded: " + str(N.load_error))
    return _MaxPoolNHWC.apply(x, tuple(k), tuple(s), tuple(p), bool(ceil_mode))
