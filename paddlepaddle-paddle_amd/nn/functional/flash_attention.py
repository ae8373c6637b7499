"""Attention functionals (reference: python/paddle/nn/functional/flash_attention.py).

Paddle's attention layout is ``[batch, seq, heads, head_dim]`` (BSHD).  On HIP tensors
``flash_attention`` / ``scaled_dot_product_attention`` run ``csrc/flash_attn.hip``: an
MFMA (16x16x32 bf16) forward with online softmax that consumes BSHD directly, and a
recompute-based backward — no [S, S] score matrix is materialised.
"""
import math

import torch
import torch.nn.functional as TF

from ...core.tensor import Tensor, _wrap as _w, _unwrap as _u
from ... import ops


def masked_attention_bhsd(q, k, v, mask, dropout_p=0.0, scale=None):
    """Explicit masked attention on [B, H, S, D] (scores -> masked fp32 softmax -> PV).

    Used for masked attention on the GPU instead of the storage layer's fused SDPA backends
    (their broadcast-mask kernels are not relied on here); every step is a plain op, so it also
    records cleanly into static Programs.  Bool masks: True = keep; float masks are additive.
    """
    sc = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    s = torch.matmul(q, k.transpose(-1, -2)).float() * sc
    if mask is not None:
        if mask.dtype == torch.bool:
            s = s.masked_fill(~mask, -1e30)
        else:
            s = s + mask.float()
    p = torch.softmax(s, -1)
    if dropout_p > 0.0:
        p = TF.dropout(p, dropout_p)
    return torch.matmul(p.to(v.dtype), v)


def _sdpa_reference(q, k, v, mask, dropout_p, causal, scale=None):
    # BSHD → BHSD for the math path
    qh, kh, vh = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    if kh.shape[1] != qh.shape[1]:  # GQA
        rep = qh.shape[1] // kh.shape[1]
        kh = kh.repeat_interleave(rep, 1)
        vh = vh.repeat_interleave(rep, 1)
    if mask is not None and (qh.is_cuda or qh.is_meta):
        if causal:
            S, Sk = qh.shape[-2], kh.shape[-2]
            cm = torch.ones(S, Sk, dtype=torch.bool, device=qh.device).tril(Sk - S)
            mask = (mask & cm) if mask.dtype == torch.bool else mask.masked_fill(~cm, float('-inf'))
        return masked_attention_bhsd(qh, kh, vh, mask, dropout_p, scale).transpose(1, 2)
    out = TF.scaled_dot_product_attention(qh, kh, vh, attn_mask=mask, dropout_p=dropout_p,
                                          is_causal=causal and mask is None, scale=scale)
    return out.transpose(1, 2)


def _attend(q, k, v, mask=None, dropout=0.0, causal=False, training=True, scale=None):
    if not training:
        dropout = 0.0
    if mask is None and dropout == 0.0 and ops.use_hip(q) and ops.flash_attn.supported(q, k, v):
        return ops.flash_attn.flash_attention(q, k, v, causal, scale)
    return _sdpa_reference(q, k, v, mask, dropout, causal, scale)


def flash_attention(query, key, value, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                    rng_name="", training=True, name=None):
    q, k, v = _u(query), _u(key), _u(value)
    out = _attend(q, k, v, None, dropout, causal, training)
    sm = None
    if return_softmax:
        s = torch.einsum('bqhd,bkhd->bhqk', q.float(), k.float()) / math.sqrt(q.shape[-1])
        if causal:
            s = s.masked_fill(torch.ones(s.shape[-2:], dtype=torch.bool, device=q.device).triu(1), float('-inf'))
        sm = _w(torch.softmax(s, -1).to(q.dtype))
    return _w(out), sm


def flash_attn_qkvpacked(qkv, dropout=0.0, causal=False, return_softmax=False, *, fixed_seed_offset=None,
                         rng_name="", training=True, name=None):
    t = _u(qkv)  # [b, s, nheads/nheads_k + 2, nheads_k, d]: groups of query heads, then k, then v
    b, s = t.shape[0], t.shape[1]
    q = t[:, :, :-2].reshape(b, s, -1, t.shape[-1])
    k, v = t[:, :, -2], t[:, :, -1]
    if (t.dim() == 5 and t.shape[2] == 3 and not return_softmax and (dropout == 0.0 or not training)
            and ops.use_hip(t) and ops.flash_attn.supported(q, k, v)):
        return _w(ops.flash_attn.flash_attention_packed(t, causal)), None
    return flash_attention(_w(q), _w(k), _w(v), dropout, causal, return_softmax, training=training)


def flash_attn_unpadded(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale,
                        dropout=0.0, causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                        training=True, name=None):
    """Variable-length attention over packed [total_tokens, heads, dim] tensors."""
    q, k, v = _u(query), _u(key), _u(value)
    cq, ck = _u(cu_seqlens_q).tolist(), _u(cu_seqlens_k).tolist()
    outs = []
    for i in range(len(cq) - 1):
        qi = q[cq[i]:cq[i + 1]].unsqueeze(0)
        ki = k[ck[i]:ck[i + 1]].unsqueeze(0)
        vi = v[ck[i]:ck[i + 1]].unsqueeze(0)
        outs.append(_attend(qi, ki, vi, None, dropout, causal, training, scale)[0])
    return _w(torch.cat(outs, 0)), None


flash_attn_varlen_qkvpacked = None


def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, training=True,
                                 name=None):
    q, k, v = _u(query), _u(key), _u(value)
    m = _u(attn_mask) if attn_mask is not None else None
    return _w(_attend(q, k, v, m, dropout_p, is_causal, training))


def flash_attention_with_sparse_mask(query, key, value, attn_mask_start_row_indices, attn_mask_start_row=0,
                                     dropout_p=0.0, is_causal=False, return_softmax=False, return_softmax_lse=False,
                                     return_seed_offset=False, training=True, name=None):
    q, k, v = _u(query), _u(key), _u(value)
    S = q.shape[1]
    rows = _u(attn_mask_start_row_indices)  # [b, h, S_k]: masked from this row downward
    r = torch.arange(S, device=q.device).view(1, 1, S, 1)
    mask = r < rows.unsqueeze(2)
    if is_causal:
        mask = mask & torch.ones(S, S, dtype=torch.bool, device=q.device).tril()
    return _w(_sdpa_reference(q, k, v, mask, dropout_p if training else 0.0, False))


def sparse_attention(query, key, value, sparse_csr_offset, sparse_csr_columns, key_padding_mask=None, attn_mask=None,
                     name=None):
    q, k, v = _u(query), _u(key), _u(value)  # [b, h, s, d]
    off, cols = _u(sparse_csr_offset), _u(sparse_csr_columns)
    B, H, S, D = q.shape
    mask = torch.zeros(B, H, S, S, dtype=torch.bool, device=q.device)
    for b in range(B):
        for h in range(H):
            o = off[b, h].tolist()
            c = cols[b, h]
            for i in range(S):
                mask[b, h, i, c[o[i]:o[i + 1]]] = True
    return _w(TF.scaled_dot_product_attention(q, k, v, attn_mask=mask))


def memory_efficient_attention(query, key, value, attn_bias=None, p=0.0, scale=None, training=True):
    q, k, v = _u(query), _u(key), _u(value)
    return _w(_attend(q, k, v, _u(attn_bias) if attn_bias is not None else None, p, False, training, scale))
