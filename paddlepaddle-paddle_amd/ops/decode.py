"""Decode-phase attention and KV-cache writes on csrc/decode_attn.hip (split-K flash decoding over a
contiguous [B, Hkv, max_len, D] or paged [num_blocks, Hkv, block_size, D] cache), with exact torch
references used on CPU and as the test oracle.

Reference: paddle/phi/kernels/fusion/gpu/masked_multihead_attention_kernel.cu,
block_multi_head_attention_kernel.cu.
"""
import math

import torch

from . import _native as N

from .workspace import workspace as _new_workspace

_DEC_WS = _new_workspace('decode_partials')


def _ws(n, dev):
    """fp32 split-K partials of the decode kernels (capture-safe: DecodeStepGraph replays keep
    the buffer they captured, ops/workspace.py)."""
    return _DEC_WS.get(n, torch.float32, dev, min_numel=1 << 16)


def _hip(*ts):
    from . import use_hip
    return all(t is None or (isinstance(t, torch.Tensor) and t.is_cuda) for t in ts) and use_hip(ts[0])


def _rows(t):
    """(tensor viewed as [rows, cols] with unit inner stride, row stride)."""
    if t.dim() == 3 and t.stride(2) == 1 and t.stride(1) == t.shape[2]:
        return t, t.stride(0)
    t = t.contiguous()
    return t, t.stride(0)


def kv_cache_write(k_new, v_new, cache_k, cache_v, pos, seq_of=None, block_tables=None, k_bias=None, v_bias=None):
    """Write rows of k_new / v_new ([R, Hkv, D]) into the cache at pos[r] (int) for sequence
    seq_of[r] (default r).  cache: contiguous [B, Hkv, L, D] or paged [nblk, Hkv, bs, D] + block_tables."""
    R, Hkv, D = k_new.shape
    pos = pos.to(torch.int32).contiguous()
    seq_of = None if seq_of is None else seq_of.to(torch.int32).contiguous()
    if _hip(k_new, v_new, cache_k, cache_v) and cache_k.is_contiguous() and cache_v.is_contiguous() and \
            k_new.dtype in (torch.bfloat16, torch.float16) and cache_k.dtype == k_new.dtype:
        kn, ks = _rows(k_new)
        vn, vs = _rows(v_new)
        if ks != vs:
            kn, vn = kn.contiguous(), vn.contiguous()
            ks = kn.stride(0)
        bt = None if block_tables is None else block_tables.to(torch.int32).contiguous()
        N.check(N.lib.pa_kv_cache_write(N.dtcode(kn.dtype), N.ptr(kn), N.ptr(vn), ks,
                                        N.ptr(None if k_bias is None else k_bias.contiguous()),
                                        N.ptr(None if v_bias is None else v_bias.contiguous()),
                                        N.ptr(cache_k), N.ptr(cache_v), N.ptr(bt),
                                        0 if bt is None else bt.shape[1], cache_k.shape[2],
                                        0 if bt is not None else cache_k.shape[2], N.ptr(seq_of), N.ptr(pos), R, Hkv,
                                        D, N.stream()), 'kv_cache_write')
        return
    kb = k_new if k_bias is None else k_new + k_bias.reshape(1, Hkv, D)
    vb = v_new if v_bias is None else v_new + v_bias.reshape(1, Hkv, D)
    for r in range(R):
        p = int(pos[r])
        if p < 0:
            continue
        b = r if seq_of is None else int(seq_of[r])
        if block_tables is None:
            cache_k[b, :, p] = kb[r].to(cache_k.dtype)
            cache_v[b, :, p] = vb[r].to(cache_v.dtype)
        else:
            bs = cache_k.shape[2]
            blk = int(block_tables[b, p // bs])
            cache_k[blk, :, p % bs] = kb[r].to(cache_k.dtype)
            cache_v[blk, :, p % bs] = vb[r].to(cache_v.dtype)


def kv_cache_write_q8(k_new, v_new, cache_k, cache_v, pos, k_quant, v_quant, seq_of=None, block_tables=None,
                      round_type=0, qmax=127.0, qmin=-127.0):
    """Quantising cache write into an int8 / uint8 cache: clip(round(x * quant_scale), qmin, qmax)
    (+128 for uint8).  k_quant / v_quant: [Hkv] (static) or [B, Hkv] (per sequence, indexed by
    seq_of[r]).  round_type 0 rounds half to even, 1 half away from zero."""
    R, Hkv, D = k_new.shape
    pos = pos.to(torch.int32).contiguous()
    seq_of = None if seq_of is None else seq_of.to(torch.int32).contiguous()
    kq, vq = k_quant.float().contiguous(), v_quant.float().contiguous()
    dyn = kq.numel() > Hkv
    if _hip(k_new, v_new, cache_k, cache_v, kq, vq) and cache_k.is_contiguous() and cache_v.is_contiguous() and \
            k_new.dtype in (torch.bfloat16, torch.float16) and cache_k.dtype in (torch.int8, torch.uint8) and \
            cache_v.dtype == cache_k.dtype:
        kn, ks = _rows(k_new)
        vn, vs = _rows(v_new)
        if ks != vs:
            kn, vn = kn.contiguous(), vn.contiguous()
            ks = kn.stride(0)
        bt = None if block_tables is None else block_tables.to(torch.int32).contiguous()
        N.check(N.lib.pa_kv_cache_write_q8(N.dtcode(kn.dtype), 3 if cache_k.dtype == torch.int8 else 4, N.ptr(kn),
                                           N.ptr(vn), ks, N.ptr(cache_k), N.ptr(cache_v), N.ptr(bt),
                                           0 if bt is None else bt.shape[1], cache_k.shape[2],
                                           0 if bt is not None else cache_k.shape[2], N.ptr(seq_of), N.ptr(pos), R,
                                           Hkv, D, N.ptr(kq), N.ptr(vq), Hkv if dyn else 0, int(round_type),
                                           float(qmax), float(qmin), N.stream()), 'kv_cache_write_q8')
        return
    zp = 128.0 if cache_k.dtype == torch.uint8 else 0.0
    sq = (torch.arange(R, device=k_new.device) if seq_of is None else seq_of).long()

    def qz(x, sc):
        s_ = sc.reshape(-1, Hkv)[sq][:, :, None] if dyn else sc.reshape(1, Hkv, 1)
        y = x.float() * s_
        y = torch.round(y) if round_type == 0 else torch.sign(y) * torch.floor(y.abs() + 0.5)
        return (y.clamp(qmin, qmax) + zp).to(cache_k.dtype)
    kk, vv = qz(k_new, kq), qz(v_new, vq)
    ok = pos >= 0
    p_, b_ = pos.long()[ok], sq[ok]
    if block_tables is None:
        cache_k[b_, :, p_] = kk[ok]
        cache_v[b_, :, p_] = vv[ok]
    else:
        bs = cache_k.shape[2]
        blk = block_tables.long()[b_, p_ // bs]
        cache_k[blk, :, p_ % bs] = kk[ok]
        cache_v[blk, :, p_ % bs] = vv[ok]


def _gather_cache(cache, b, L, block_tables):
    """[Hkv, L, D] view of sequence b's first L positions."""
    if block_tables is None:
        return cache[b, :, :L]
    bs = cache.shape[2]
    nb = (L + bs - 1) // bs
    blocks = cache[block_tables[b, :nb].long()]           # [nb, Hkv, bs, D]
    return blocks.permute(1, 0, 2, 3).reshape(cache.shape[1], nb * bs, cache.shape[3])[:, :L]


def decode_attention_ref(q, cache_k, cache_v, lens, block_tables=None, mask=None, q_bias=None, scale=None):
    """fp32 reference: q [B, Hq, D] attends over positions [0, lens[b]) of its cache."""
    B, Hq, D = q.shape
    Hkv = cache_k.shape[1]
    G = Hq // Hkv
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    qq = q.float() + (0 if q_bias is None else q_bias.float().reshape(1, Hq, D))
    out = torch.zeros(B, Hq, D, dtype=torch.float32, device=q.device)
    for b in range(B):
        L = int(lens[b])
        if L <= 0:
            continue
        k = _gather_cache(cache_k, b, L, block_tables).float().repeat_interleave(G, 0)  # [Hq, L, D]
        v = _gather_cache(cache_v, b, L, block_tables).float().repeat_interleave(G, 0)
        s = torch.einsum('hd,hld->hl', qq[b], k) * scale
        if mask is not None:
            s = s + mask[b, :L].float()
        out[b] = torch.einsum('hl,hld->hd', torch.softmax(s, -1), v)
    return out.to(q.dtype)


def _dequant_cache(cache, sc, zero_pt, dtype):
    """8-bit cache -> (x - zero_pt) * scale; sc [Hkv] or [B, Hkv] (contiguous caches only)."""
    s_ = sc.float().reshape(-1, cache.shape[1]) if sc.dim() > 1 else sc.float().reshape(1, -1)
    return ((cache.float() - zero_pt) * s_[:, :, None, None]).to(dtype)


def decode_attention(q, cache_k, cache_v, lens, block_tables=None, mask=None, q_bias=None, scale=None,
                     k_dequant=None, v_dequant=None):
    """One decode step: q [B, Hq, D] (rows may be strided views of a fused qkv) over the cache.
    lens: int [B] positions to attend (new token included); mask: additive [B, >= max_len] fp32.
    8-bit caches (int8: round(x * quant_scale); uint8: that + 128) take fp32 dequant scales
    k_dequant / v_dequant of shape [Hkv] (static) or [B, Hkv] (dynamic, per sequence) and are
    dequantised inside the kernel (bf16 queries, D 64 / 128)."""
    B, Hq, D = q.shape
    Hkv = cache_k.shape[1]
    scale = 1.0 / math.sqrt(D) if scale is None else float(scale)
    G = Hq // Hkv if Hkv else 0
    q8 = cache_k.dtype in (torch.int8, torch.uint8)
    if q8:
        if k_dequant is None or v_dequant is None:
            raise ValueError("an 8-bit KV cache needs k_dequant / v_dequant scales")
        ks = k_dequant.float().contiguous()
        vs = v_dequant.float().contiguous()
        if ks.numel() not in (Hkv, B * Hkv) or vs.numel() != ks.numel():
            raise ValueError(f"dequant scales must have {Hkv} or {B}x{Hkv} entries, got {ks.numel()} / {vs.numel()}")
        zp = 128.0 if cache_k.dtype == torch.uint8 else 0.0
        hip_ok = (_hip(q, cache_k, cache_v, ks, vs) and Hq % Hkv == 0 and cache_k.is_contiguous()
                  and cache_v.is_contiguous() and cache_v.dtype == cache_k.dtype and q.dtype == torch.bfloat16
                  and D in (64, 128) and N.lib.pa_decode_ok(N.dtcode(q.dtype), D, G))
        if not hip_ok:
            if block_tables is not None:  # gather the pages first, then dequantise
                nb, bs = block_tables.shape[1], cache_k.shape[2]
                pg = block_tables.long()
                cache_k = cache_k[pg].permute(0, 2, 1, 3, 4).reshape(B, Hkv, nb * bs, D)
                cache_v = cache_v[pg].permute(0, 2, 1, 3, 4).reshape(B, Hkv, nb * bs, D)
                block_tables = None
            kd = _dequant_cache(cache_k, ks.reshape(-1, Hkv) if ks.numel() > Hkv else ks, zp, q.dtype)
            vd = _dequant_cache(cache_v, vs.reshape(-1, Hkv) if vs.numel() > Hkv else vs, zp, q.dtype)
            if kd.shape[0] != B:
                kd, vd = kd.expand(B, -1, -1, -1), vd.expand(B, -1, -1, -1)
            return decode_attention_ref(q, kd, vd, lens, None, mask, q_bias, scale)
    elif not (_hip(q, cache_k, cache_v) and Hq % Hkv == 0 and cache_k.is_contiguous() and cache_v.is_contiguous()
              and q.dtype == cache_k.dtype and N.lib.pa_decode_ok(N.dtcode(q.dtype), D, G)):
        return decode_attention_ref(q, cache_k, cache_v, lens, block_tables, mask, q_bias, scale)
    qr, qs = _rows(q)
    lens = lens.to(torch.int32).contiguous()
    bt = None if block_tables is None else block_tables.to(torch.int32).contiguous()
    span = bt.shape[1] * cache_k.shape[2] if bt is not None else cache_k.shape[2]
    msk = None if mask is None else mask.float().contiguous()
    nsplit = N.lib.pa_decode_nsplit(B, Hkv, span)
    out = torch.empty(B, Hq, D, dtype=q.dtype, device=q.device)
    ws = _ws(B * Hq * nsplit * (D + 2), q.device) if nsplit > 1 else None
    qb = N.ptr(None if q_bias is None else q_bias.contiguous())
    common = (N.ptr(cache_k), N.ptr(cache_v), N.ptr(bt), 0 if bt is None else bt.shape[1], cache_k.shape[2],
              0 if bt is not None else cache_k.shape[2], N.ptr(lens), N.ptr(msk),
              0 if msk is None else msk.stride(0), N.ptr(out), Hq * D, N.ptr(ws), B, Hq, Hkv, D, nsplit, scale)
    if q8:
        N.check(N.lib.pa_decode_attn_q8(3 if cache_k.dtype == torch.int8 else 4, N.ptr(qr), qs, qb, *common,
                                        N.ptr(ks), N.ptr(vs), Hkv if ks.numel() > Hkv else 0, N.stream()),
                'decode_attn_q8')
    else:
        N.check(N.lib.pa_decode_attn(N.dtcode(q.dtype), N.ptr(qr), qs, qb, *common, N.stream()), 'decode_attn')
    return out
