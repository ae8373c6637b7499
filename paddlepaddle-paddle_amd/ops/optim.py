"""Fused AdamW over flat buffers on csrc/embed_rope_optim.hip.

Reference: paddle/phi/kernels/gpu/adamw_kernel.cu (multi_precision: fp32 master weight,
low-precision model copy written in the same pass).  One launch updates an entire flat
parameter shard: master (fp32), m, v, and the bf16 model parameters.
"""
import torch

from . import _native as N


def adamw_flat(master, grad, m, v, lowp, lr, beta1, beta2, eps, weight_decay, beta1_pow, beta2_pow, lr_tensor=None,
               grad_scale=None, pows=None):
    """pows (optional): device fp32 [beta1_pow, beta2_pow] read by the kernel instead of the host
    values (the caller advances it on the device, so a captured step replays with fresh powers)."""
    n = master.numel()
    assert grad.numel() == n and m.numel() == n and v.numel() == n
    pd = -1 if lowp is None else N.dtcode(lowp.dtype)
    N.check(N.lib.pa_adamw(N.ptr(master), N.ptr(grad), N.ptr(m), N.ptr(v), N.ptr(lowp), n, N.ptr(lr_tensor),
                           float(lr), beta1, beta2, eps, weight_decay, float(beta1_pow), float(beta2_pow),
                           N.ptr(grad_scale), N.ptr(pows), N.dtcode(grad.dtype), pd, N.stream()), 'adamw')


def sumsq(x):
    """Sum of squares of a flat buffer as a 0-d fp32 tensor (two-stage, deterministic)."""
    parts = torch.empty(N.lib.pa_sumsq_parts(), dtype=torch.float32, device=x.device)
    N.check(N.lib.pa_sumsq(N.ptr(x), x.numel(), N.ptr(parts), N.dtcode(x.dtype), N.stream()), 'sumsq')
    return parts.sum()


def momentum_flat(master, grad, velocity, lowp, lr, mu, l2=0.0, rescale=1.0, nesterov=False, grad_scale=None,
                  lr_tensor=None):
    """Fused momentum over flat buffers (csrc/embed_rope_optim.hip momentum_kernel).  ``lr_tensor``: a
    device fp32 [1] learning rate read by the kernel instead of ``lr`` (captured steps)."""
    n = master.numel()
    assert grad.numel() == n and velocity.numel() == n
    pd = -1 if lowp is None else N.dtcode(lowp.dtype)
    N.check(N.lib.pa_momentum(N.ptr(master), N.ptr(grad), N.ptr(velocity), N.ptr(lowp), n, N.ptr(lr_tensor), float(lr), float(mu),
                              float(l2), float(rescale), int(bool(nesterov)), N.ptr(grad_scale), N.dtcode(grad.dtype),
                              pd, N.stream()), 'momentum')
