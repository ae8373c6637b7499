"""Loss-scaling kernels (csrc/amp.hip): multi-tensor check_finite_and_unscale and the dynamic
loss-scale update on device-resident state — the reference's ``check_finite_and_unscale`` /
``update_loss_scaling`` ops (paddle/phi/kernels/gpu/amp_kernel.cu, inserted by
python/paddle/static/amp/decorator.py:548,589).  CPU tensors take the same math in torch."""
import ctypes

import torch

from . import _native as N

_MAXT = 48


def check_finite_and_unscale_(grads, scale, found_inf):
    """grads[i] *= 1 / scale in place; found_inf (fp32 [1]) is set to 1 when any gradient holds an
    inf / nan (it is NOT cleared: zero it once per step).  ``scale``: device fp32 [1] tensor."""
    grads = [g for g in grads if g is not None and g.numel() > 0]
    if not grads:
        return found_inf
    if grads[0].is_cuda and (N.lib is not None or N._load() is not None):
        by = [g if g.is_contiguous() else None for g in grads]
        rest = [g for g, b in zip(grads, by) if b is None]
        ok = [b for b in by if b is not None and b.dtype in (torch.float32, torch.bfloat16, torch.float16)]
        rest += [b for b in by if b is not None and b.dtype not in (torch.float32, torch.bfloat16, torch.float16)]
        for i in range(0, len(ok), _MAXT):
            part = ok[i:i + _MAXT]
            n = len(part)
            ptrs = (ctypes.c_void_p * n)(*[g.data_ptr() for g in part])
            numel = (ctypes.c_longlong * n)(*[g.numel() for g in part])
            dts = (ctypes.c_int * n)(*[N.dtcode(g.dtype) for g in part])
            N.check(N.lib.pa_amp_check_unscale(ctypes.cast(ptrs, ctypes.c_void_p), ctypes.cast(numel, ctypes.c_void_p),
                                               ctypes.cast(dts, ctypes.c_void_p), n, N.ptr(scale), N.ptr(found_inf),
                                               N.stream()), 'amp_check_unscale')
        grads = rest
    inv = 1.0 / scale.float()
    for g in grads:
        bad = ~torch.isfinite(g).all()
        found_inf.copy_(torch.where(bad, torch.ones_like(found_inf), found_inf))
        g.mul_(inv.to(g.dtype) if g.is_floating_point() else inv)
    return found_inf


def update_loss_scaling_(found_inf, scale, good, bad, incr_every_n_steps, decr_every_n_nan_or_inf, incr_ratio,
                         decr_ratio, min_scale=1.0):
    """The dynamic loss-scale rule on device scalars (fp32 [1] each), no host round trip."""
    if scale.is_cuda and (N.lib is not None or N._load() is not None):
        N.check(N.lib.pa_amp_update_scale(N.ptr(scale), N.ptr(good), N.ptr(bad), N.ptr(found_inf),
                                          int(incr_every_n_steps), int(decr_every_n_nan_or_inf), float(incr_ratio),
                                          float(decr_ratio), float(min_scale), N.stream()), 'amp_update_scale')
        return scale
    f = bool(found_inf.item() != 0)
    if f:
        good.zero_()
        bad.add_(1)
        if bad.item() >= decr_every_n_nan_or_inf:
            scale.copy_(torch.clamp(scale * decr_ratio, min=min_scale))
            bad.zero_()
    else:
        bad.zero_()
        good.add_(1)
        if good.item() >= incr_every_n_steps:
            ns = scale * incr_ratio
            scale.copy_(torch.where(torch.isfinite(ns), ns, scale))
            good.zero_()
    return scale
