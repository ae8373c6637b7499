"""Flash attention (BSHD) on csrc/flash_attn.hip — MFMA forward + recompute backward.

Reference: paddle/phi/kernels/gpu/flash_attn_kernel.cu / flash_attn_grad_kernel.cu.
"""
import math

import torch

from . import _native as N


def supported(q, k, v):
    return (q.dim() == 4 and q.dtype in (torch.bfloat16, torch.float16) and k.dtype == q.dtype and v.dtype == q.dtype
            and q.shape[-1] in (64, 128) and k.shape[-1] == q.shape[-1] and v.shape[-1] == q.shape[-1]
            and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1
            and k.shape[2] > 0 and q.shape[2] % k.shape[2] == 0 and k.shape == v.shape
            and all(s % 8 == 0 for t in (q, k, v) for s in t.stride()[:3]))


def _fwd(q, k, v, causal, scale):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    o = torch.empty(B, Sq, Hq, D, dtype=q.dtype, device=q.device)
    lse = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
    N.check(N.lib.pa_flash_fwd(N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(lse), B, Sq, Sk, Hq, Hk, D,
                               N.strides3(q), N.strides3(k), N.strides3(v), N.strides3(o), scale, int(causal),
                               N.dtcode(q.dtype), N.stream()), 'flash_fwd')
    return o, lse


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = _fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        B, Sq, Hq, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        if do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]):
            do = do.contiguous()
        dq = torch.empty(B, Sq, Hq, D, dtype=q.dtype, device=q.device)
        dk = torch.empty(B, Sk, Hq, D, dtype=q.dtype, device=q.device)
        dv = torch.empty(B, Sk, Hq, D, dtype=q.dtype, device=q.device)
        delta = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
        N.check(N.lib.pa_flash_bwd(N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(do), N.ptr(lse), N.ptr(delta),
                                   N.ptr(dq), N.ptr(dk), N.ptr(dv), B, Sq, Sk, Hq, Hk, D, N.strides3(q), N.strides3(k),
                                   N.strides3(v), N.strides3(o), N.strides3(do), N.strides3(dq), N.strides3(dk),
                                   N.strides3(dv), ctx.scale, int(ctx.causal), N.dtcode(q.dtype), N.stream()),
                'flash_bwd')
        if Hq != Hk:  # GQA: sum the per-q-head dK/dV over each kv group
            dk = dk.view(B, Sk, Hk, Hq // Hk, D).sum(3)
            dv = dv.view(B, Sk, Hk, Hq // Hk, D).sum(3)
        return dq, dk, dv, None, None


class _FlashAttnPacked(torch.autograd.Function):
    """qkv: [B, S, 3, H, D].  The backward writes dQ/dK/dV straight into one packed gradient
    (the kernels take output strides), so the packed projection's grad needs no zero-fill,
    slice copies or sums — three full-size passes per layer that per-view grads would cost."""

    @staticmethod
    def forward(ctx, qkv, causal, scale):
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        o, lse = _fwd(q, k, v, causal, scale)
        ctx.save_for_backward(qkv, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse = ctx.saved_tensors
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        B, S, H, D = q.shape
        if do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]):
            do = do.contiguous()
        dqkv = torch.empty(B, S, 3, H, D, dtype=qkv.dtype, device=qkv.device)
        dq, dk, dv = dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2]
        delta = torch.empty(B, H, S, dtype=torch.float32, device=q.device)
        N.check(N.lib.pa_flash_bwd(N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(do), N.ptr(lse), N.ptr(delta),
                                   N.ptr(dq), N.ptr(dk), N.ptr(dv), B, S, S, H, H, D, N.strides3(q), N.strides3(k),
                                   N.strides3(v), N.strides3(o), N.strides3(do), N.strides3(dq), N.strides3(dk),
                                   N.strides3(dv), ctx.scale, int(ctx.causal), N.dtcode(q.dtype), N.stream()),
                'flash_bwd')
        return dqkv, None, None


def flash_attention_packed(qkv, causal=False, scale=None):
    """qkv: [B, S, 3, H, D] with unit last-dim stride."""
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    return _FlashAttnPacked.apply(qkv, bool(causal), float(scale))


def flash_attention(q, k, v, causal=False, scale=None):
    """q: [B, Sq, Hq, D], k/v: [B, Sk, Hk, D] (any strides with unit last-dim stride)."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return _FlashAttn.apply(q, k, v, bool(causal), float(scale))


def flash_attention_with_lse(q, k, v, causal=False, scale=None):
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return _fwd(q, k, v, causal, scale)
