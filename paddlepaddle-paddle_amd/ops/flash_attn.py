"""Flash attention (BSHD) on csrc/flash_attn.hip — MFMA forward + recompute backward.

Reference: paddle/phi/kernels/gpu/flash_attn_kernel.cu / flash_attn_grad_kernel.cu.
"""
from ..framework.flags import pa_flag  # noqa: E402
import math
import os

import torch

from . import _native as N


# head dims with native tiles: 64 / 128 (csrc/flash_attn.hip), 96 / 256 (csrc/flash_attn_wide.hip)
HEAD_DIMS = (64, 96, 128, 256)


def tiled_head_dim(D):
    """The smallest natively tiled head dim >= D (operands are zero-padded to it), or None."""
    for t in HEAD_DIMS:
        if D <= t:
            return t
    return None


def supported_ex(q, k, v):
    """The extended kernels (mask / dropout / varlen) take the same operand contract."""
    return supported(q, k, v)


def supported(q, k, v):
    return (q.dim() == 4 and q.dtype in (torch.bfloat16, torch.float16) and k.dtype == q.dtype and v.dtype == q.dtype
            and q.shape[-1] in HEAD_DIMS and k.shape[-1] == q.shape[-1] and v.shape[-1] == q.shape[-1]
            and q.stride(-1) == 1 and k.stride(-1) == 1 and v.stride(-1) == 1
            and k.shape[2] > 0 and q.shape[2] % k.shape[2] == 0 and k.shape == v.shape
            and all(s % 8 == 0 for t in (q, k, v) for s in t.stride()[:3]))


# Backward with a materialised dS (csrc/flash_attn_ds.hip): delta pass, dK/dV kernel that also
# stores dS^T, dQ = dS K from it — instead of a second kernel recomputing S and dP.  The dS^T
# workspace (B * Hq * Sk * ceil(Sq / 128) * 128 elements, 0.5 GB for GPT-3 1.3B's attention) is
# kept per device and reused by every layer.  Default: head_dim 128 (B16 S1024 H16 causal
# fwd+bwd 0.720 -> 0.651 ms, GPT-3 1.3B step 124.4k -> 125.7k tok/s, profiles/r4e_attn_ds_ab.log);
# head_dim 64 stays on the recompute pair (1.04 -> 1.24 ms there: its dQ recompute is cheaper than
# the dS round trip).  PADDLE_AMD_FA_DS_BWD=0 / 1: off / also for head_dim 64.
_ds_env = (pa_flag('fa_ds_bwd') or None)
_ds_bwd = [None if _ds_env is None else _ds_env != '0']  # None: automatic (head_dim 128)
# bounded: a dS^T image above PADDLE_AMD_FA_DS_WS_MB (default 8 GiB) takes the recompute kernels
from .workspace import workspace as _workspace
_DS_WS = _workspace('flash_ds', int(pa_flag('fa_ds_ws_mb')) << 20)


def set_ds_backward(on):
    """True: every supported head dim, False: off, None: automatic (head_dim 128).  Returns the old."""
    old = _ds_bwd[0]
    _ds_bwd[0] = None if on is None else bool(on)
    return old


def _ds_ok(D, dt):
    if dt not in (torch.bfloat16, torch.float16):
        return False
    on = _ds_bwd[0]
    return D == 128 if on is None else (on and D in (64, 128))


def _ds_ws(B, Hq, Sq, Sk, dtype, device):
    """The shared dS^T workspace, or None when it would exceed the bound."""
    n = int(N.lib.pa_flash_ds_ws_elems(B, Hq, Sq, Sk))
    if not _DS_WS.fits(n, dtype):
        return None
    return _DS_WS.get(n, dtype, device)


def _bwd_call(q, k, v, o, do, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, D, scale, causal, cu_q=None, cu_k=None,
              total=0, m=None, mb=0, mh=0, mq=0, mf=0, p_drop=0.0, seed=0, rows=None, rb=0, rh=0, ex=False):
    """The backward launch sequence: dS path when enabled, else the recompute kernels
    (pa_flash_bwd, or pa_flash_bwd_ex when any extended feature is in use)."""
    mall = _mask_all(m, mh, mq)
    st = (N.strides3(q), N.strides3(k), N.strides3(v), N.strides3(o), N.strides3(do), N.strides3(dq),
          N.strides3(dk), N.strides3(dv))
    ws = _ds_ws(B, Hq, Sq, Sk, q.dtype, q.device) if _ds_ok(D, q.dtype) else None
    if ws is not None:
        N.check(N.lib.pa_flash_bwd_ds(N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(do), N.ptr(lse), N.ptr(delta),
                                      N.ptr(dq), N.ptr(dk), N.ptr(dv), N.ptr(ws), B, Sq, Sk, Hq, Hk, D, *st, scale,
                                      int(causal), N.dtcode(q.dtype), N.ptr(cu_q), N.ptr(cu_k), total, N.ptr(m), mb,
                                      mh, mq, mf, float(p_drop), seed & 0xFFFFFFFF, 0, N.ptr(rows), rb, rh,
                                      N.ptr(mall), N.stream()), 'flash_bwd_ds')
    elif ex:
        N.check(N.lib.pa_flash_bwd_ex(N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(do), N.ptr(lse), N.ptr(delta),
                                      N.ptr(dq), N.ptr(dk), N.ptr(dv), B, Sq, Sk, Hq, Hk, D, *st, scale, int(causal),
                                      N.dtcode(q.dtype), N.ptr(cu_q), N.ptr(cu_k), total, N.ptr(m), mb, mh, mq, mf,
                                      float(p_drop), seed & 0xFFFFFFFF, 0, N.ptr(rows), rb, rh, N.ptr(mall),
                                      N.stream()), 'flash_bwd_ex')
    else:
        N.check(N.lib.pa_flash_bwd(N.ptr(q), N.ptr(k), N.ptr(v), N.ptr(o), N.ptr(do), N.ptr(lse), N.ptr(delta),
                                   N.ptr(dq), N.ptr(dk), N.ptr(dv), B, Sq, Sk, Hq, Hk, D, *st, scale, int(causal),
                                   N.dtcode(q.dtype), N.stream()), 'flash_bwd')


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
        _bwd_call(q, k, v, o, do, lse, delta, dq, dk, dv, B, Sq, Sk, Hq, Hk, D, ctx.scale, ctx.causal)
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
        _bwd_call(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, S, H, H, D, ctx.scale, ctx.causal)
        return dqkv, None, None


class _QKVRopeFlash(torch.autograd.Function):
    """Fused-QKV projection output [B, S, Hq + 2 Hkv, D] -> RoPE on the q / k head slices ->
    causal flash attention.  Forward: the rotated q / k are written straight from the strided
    slices (no .contiguous() copies), v is attended in place.  Backward: dQ / dK / dV land
    directly in one packed gradient (MHA; GQA sums the per-q-head dK / dV into it) and dQ / dK are
    rotated back in place — no zero-filled per-slice gradients, adds or concatenation."""

    @staticmethod
    def forward(ctx, qkv, cos, sin, pos, nh, nkv, causal, scale):
        from . import rope
        B, S, Ht, D = qkv.shape
        q = torch.empty(B, S, nh, D, dtype=qkv.dtype, device=qkv.device)
        k = torch.empty(B, S, nkv, D, dtype=qkv.dtype, device=qkv.device)
        rope.rope_rows(qkv[:, :, :nh], q, cos, sin, pos)
        rope.rope_rows(qkv[:, :, nh:nh + nkv], k, cos, sin, pos)
        v = qkv[:, :, nh + nkv:]
        o, lse = _fwd(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, qkv, o, lse, cos, sin, pos)
        ctx.cfg = (nh, nkv, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        from . import rope
        q, k, qkv, o, lse, cos, sin, pos = ctx.saved_tensors
        nh, nkv, causal, scale = ctx.cfg
        B, S, Ht, D = qkv.shape
        v = qkv[:, :, nh + nkv:]
        if do.stride(-1) != 1 or any(s_ % 8 for s_ in do.stride()[:3]):
            do = do.contiguous()
        dqkv = torch.empty(B, S, Ht, D, dtype=qkv.dtype, device=qkv.device)
        dq, dk, dv = dqkv[:, :, :nh], dqkv[:, :, nh:nh + nkv], dqkv[:, :, nh + nkv:]
        delta = torch.empty(B, nh, S, dtype=torch.float32, device=qkv.device)
        if nh == nkv:
            _bwd_call(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, S, nh, nkv, D, scale, causal)
        else:  # GQA: per-q-head dK / dV, summed over each kv group into the packed slices
            dkh = torch.empty(B, S, nh, D, dtype=qkv.dtype, device=qkv.device)
            dvh = torch.empty(B, S, nh, D, dtype=qkv.dtype, device=qkv.device)
            _bwd_call(q, k, v, o, do, lse, delta, dq, dkh, dvh, B, S, S, nh, nkv, D, scale, causal)
            dk.copy_(dkh.view(B, S, nkv, nh // nkv, D).sum(3))
            dv.copy_(dvh.view(B, S, nkv, nh // nkv, D).sum(3))
        rope.rope_rows(dq, dq, cos, sin, pos, sign=-1.0)
        rope.rope_rows(dk, dk, cos, sin, pos, sign=-1.0)
        return dqkv, None, None, None, None, None, None, None


def qkv_rope_flash_ok(qkv, nh, nkv):
    from . import rope
    if qkv.dim() != 4 or not qkv.is_contiguous() or qkv.shape[2] != nh + 2 * nkv or nh % nkv:
        return False
    if not rope.rows_ok(qkv[:, :, :nh]) or qkv.dtype not in (torch.bfloat16, torch.float16):
        return False
    return supported(qkv[:, :, :nh], qkv[:, :, nh:nh + nkv], qkv[:, :, nh + nkv:])


def qkv_rope_flash(qkv, nh, nkv, cos, sin, pos=None, causal=True, scale=None):
    """Flash attention of RoPE'd q / k taken from a fused QKV projection output
    [B, S, nh + 2 nkv, D] (``qkv_rope_flash_ok``); cos / sin: [S_max, D/2] fp32 tables;
    pos: optional [B, S] int64 positions.  Returns o [B, S, nh, D]."""
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    p = pos.contiguous().to(torch.int64) if pos is not None else None
    return _QKVRopeFlash.apply(qkv, cos, sin, p, int(nh), int(nkv), bool(causal), float(scale))


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


# ------------------------------------------------------------------ masks, dropout, varlen
def _mask_args(mask, B, H, Sq, Sk, dtype):
    """(tensor, mb, mh, mq, is_f32) for an additive / bool mask broadcastable to [B, H, Sq, Sk]."""
    if mask is None:
        return None, 0, 0, 0, 0
    m = mask
    if m.dtype == torch.bool:
        m = torch.zeros(m.shape, dtype=dtype, device=m.device).masked_fill(~m, float('-inf'))
    elif m.dtype not in (torch.float32, dtype):
        m = m.float()
    while m.dim() < 4:
        m = m.unsqueeze(0)
    if m.stride(-1) != 1:
        m = m.contiguous()
    m = m.expand(B, H, Sq, Sk)
    st = m.stride()
    return m, st[0], st[1], st[2], int(m.dtype == torch.float32)


def _mask_all(m, mh, mq):
    """[B] int32 device flags for a key-only mask (constant over heads and queries): 1 where the
    mask keeps every key of the batch entry (an unpadded sequence), so the kernels skip its
    per-element loads; None for other masks.  No host synchronisation."""
    if m is None or mh != 0 or mq != 0:
        return None
    return (m[:, 0, 0, :] == 0).all(-1).to(torch.int32)


def _rows_args(rows, B, H, Sk):
    """(tensor, rb, rh) for flashmask start-row indices broadcastable to [B, H, Sk] (int32)."""
    if rows is None:
        return None, 0, 0
    r = rows.to(torch.int32)
    while r.dim() < 3:
        r = r.unsqueeze(0)
    if r.stride(-1) != 1:
        r = r.contiguous()
    r = r.expand(B, H, Sk)
    return r, r.stride(0), r.stride(1)


def _seed():
    from ..device.cuda.graphs import host_rng_guard
    host_rng_guard('flash attention dropout')
    return int(torch.randint(0, 2 ** 31 - 1, (1,)).item())


def _fwd_ex(q, k, v, causal, scale, mask, p_drop, seed, cu_q, cu_k, max_q, max_k, rows=None):
    if cu_q is None:
        B, Sq, Hq, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        total = 0
        o = torch.empty(B, Sq, Hq, D, dtype=q.dtype, device=q.device)
        lse = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
        qv, kv, vv, ov = q, k, v, o
    else:  # packed [total, H, D]
        total, Hq, D = q.shape
        Hk = k.shape[1]
        B, Sq, Sk = cu_q.numel() - 1, max_q, max_k
        # zeros: rows outside every sequence (padded varlen layouts) read back as 0
        o = torch.zeros(total, Hq, D, dtype=q.dtype, device=q.device)
        lse = torch.empty(Hq, total, dtype=torch.float32, device=q.device)
        qv, kv, vv, ov = q.unsqueeze(0), k.unsqueeze(0), v.unsqueeze(0), o.unsqueeze(0)
    m, mb, mh, mq, mf = _mask_args(mask, B, Hq, Sq, Sk, q.dtype)
    rows, rb, rh = _rows_args(rows, B, Hq, Sk)
    mall = _mask_all(m, mh, mq)
    N.check(N.lib.pa_flash_fwd_ex(N.ptr(qv), N.ptr(kv), N.ptr(vv), N.ptr(ov), N.ptr(lse), B, Sq, Sk, Hq, Hk, D,
                                  N.strides3(qv), N.strides3(kv), N.strides3(vv), N.strides3(ov), scale, int(causal),
                                  N.dtcode(q.dtype), N.ptr(cu_q), N.ptr(cu_k), total, N.ptr(m), mb, mh, mq, mf,
                                  float(p_drop), seed & 0xFFFFFFFF, 0, N.ptr(rows), rb, rh, N.ptr(mall), N.stream()),
            'flash_fwd_ex')
    return o, lse


class _FlashAttnEx(torch.autograd.Function):
    """Flash attention with an additive/bool mask, in-kernel dropout and/or varlen packing."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, mask, p_drop, cu_q, cu_k, max_q, max_k, rows):
        seed = _seed() if p_drop > 0 else 0
        o, lse = _fwd_ex(q, k, v, causal, scale, mask, p_drop, seed, cu_q, cu_k, max_q, max_k, rows)
        ctx.save_for_backward(q, k, v, o, lse, mask, cu_q, cu_k, rows)
        ctx.args = (causal, scale, p_drop, seed, max_q, max_k)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, mask, cu_q, cu_k, rows = ctx.saved_tensors
        causal, scale, p_drop, seed, max_q, max_k = ctx.args
        if do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:-1]):
            do = do.contiguous()
        alloc = torch.empty if cu_q is None else torch.zeros  # varlen: rows outside every sequence
        dq = alloc(q.shape, dtype=q.dtype, device=q.device)
        Hq, Hk = q.shape[-2], k.shape[-2]
        kshape = list(k.shape)
        kshape[-2] = Hq
        dk = alloc(kshape, dtype=q.dtype, device=q.device)
        dv = alloc(kshape, dtype=q.dtype, device=q.device)
        if cu_q is None:
            B, Sq, _, D = q.shape
            Sk = k.shape[1]
            total = 0
            delta = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
            views = (q, k, v, o, do, dq, dk, dv)
        else:
            total, _, D = q.shape
            B, Sq, Sk = cu_q.numel() - 1, max_q, max_k
            delta = torch.empty(Hq, total, dtype=torch.float32, device=q.device)
            views = tuple(t.unsqueeze(0) for t in (q, k, v, o, do, dq, dk, dv))
        qv, kv, vv, ov, dov, dqv, dkv, dvv = views
        m, mb, mh, mq, mf = _mask_args(mask, B, Hq, Sq, Sk, q.dtype)
        rows, rb, rh = _rows_args(rows, B, Hq, Sk)
        _bwd_call(qv, kv, vv, ov, dov, lse, delta, dqv, dkv, dvv, B, Sq, Sk, Hq, Hk, D, scale, causal, cu_q, cu_k, total,
                  m, mb, mh, mq, mf, p_drop, seed, rows, rb, rh, ex=True)
        if Hq != Hk:
            dk = dk.unflatten(-2, (Hk, Hq // Hk)).sum(-2)
            dv = dv.unflatten(-2, (Hk, Hq // Hk)).sum(-2)
        return dq, dk, dv, None, None, None, None, None, None, None, None, None


def flash_attention_ex(q, k, v, causal=False, scale=None, mask=None, dropout=0.0, cu_seqlens_q=None,
                       cu_seqlens_k=None, max_seqlen_q=None, max_seqlen_k=None, start_rows=None):
    """q/k/v [B, S, H, D] (or packed [total, H, D] with int32 cu_seqlens); mask broadcastable to
    [B, Hq, Sq, Sk] (additive, or bool = keep); dropout on the attention probabilities;
    start_rows [B, H|1, Sk] int32 flashmask indices (key k masked for queries >= start_rows[k])."""
    if mask is not None and start_rows is not None:
        raise ValueError("flash_attention_ex: pass either a dense mask or start_rows, not both")
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    cq = None if cu_seqlens_q is None else cu_seqlens_q.to(device=q.device, dtype=torch.int32).contiguous()
    ck = None if cu_seqlens_k is None else cu_seqlens_k.to(device=q.device, dtype=torch.int32).contiguous()
    if cq is not None and (max_seqlen_q is None or max_seqlen_k is None):
        max_seqlen_q = int((cq[1:] - cq[:-1]).max())
        max_seqlen_k = int((ck[1:] - ck[:-1]).max())
    return _FlashAttnEx.apply(q, k, v, bool(causal), float(scale), mask, float(dropout), cq, ck, max_seqlen_q,
                              max_seqlen_k, start_rows)


class _FlashAttnPackedEx(torch.autograd.Function):
    """Packed qkv [B, S, 3, H, D] with in-kernel dropout (and/or a mask): the training path of
    GPT with attention dropout; dQ/dK/dV land straight in one packed gradient as in
    _FlashAttnPacked."""

    @staticmethod
    def forward(ctx, qkv, causal, scale, mask, p_drop):
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        seed = _seed() if p_drop > 0 else 0
        o, lse = _fwd_ex(q, k, v, causal, scale, mask, p_drop, seed, None, None, None, None)
        ctx.save_for_backward(qkv, o, lse, mask)
        ctx.args = (causal, scale, p_drop, seed)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, mask = ctx.saved_tensors
        causal, scale, p_drop, seed = ctx.args
        q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
        B, S, H, D = q.shape
        if do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]):
            do = do.contiguous()
        dqkv = torch.empty(B, S, 3, H, D, dtype=qkv.dtype, device=qkv.device)
        dq, dk, dv = dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2]
        delta = torch.empty(B, H, S, dtype=torch.float32, device=q.device)
        m, mb, mh, mq, mf = _mask_args(mask, B, H, S, S, q.dtype)
        _bwd_call(q, k, v, o, do, lse, delta, dq, dk, dv, B, S, S, H, H, D, scale, causal, None, None, 0, m, mb, mh, mq,
                  mf, p_drop, seed, None, 0, 0, ex=True)
        return dqkv, None, None, None, None


def flash_attention_packed_ex(qkv, causal=False, scale=None, mask=None, dropout=0.0):
    if scale is None:
        scale = 1.0 / math.sqrt(qkv.shape[-1])
    return _FlashAttnPackedEx.apply(qkv, bool(causal), float(scale), mask, float(dropout))
