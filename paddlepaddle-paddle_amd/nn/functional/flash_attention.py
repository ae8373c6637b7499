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
from ...core.amp_dispatch import amp_op as _amp_op


def masked_attention_bhsd(q, k, v, mask, dropout_p=0.0, scale=None):
    """Explicit masked attention on [B, H, S, D] (scores -> masked fp32 softmax -> PV).

    Used for masked attention on the GPU instead of the storage layer's fused SDPA backends
    (their broadcast-mask kernels are not relied on here); every step is a plain op, so it also
    records cleanly into static Programs.  Bool masks: True = keep; float masks are additive.
    """
    sc = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    s = ops.matmul.matmul(q, k.transpose(-1, -2)).float() * sc
    if mask is not None:
        if mask.dtype == torch.bool:
            s = s.masked_fill(~mask, -1e30)
        else:
            s = s + mask.float()
    p = torch.softmax(s, -1)
    if dropout_p > 0.0:
        p = TF.dropout(p, dropout_p)
    return ops.matmul.matmul(p.to(v.dtype), v)


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


def _pad_head(q, k, v):
    """Head dims the kernels do not tile (e.g. 80, 192) are zero-padded to the next tiled one
    (64 / 96 / 128 / 256): the extra q·k terms are 0 and the extra output columns are sliced off."""
    D = q.shape[-1]
    Dp = ops.flash_attn.tiled_head_dim(D) or D
    if Dp == D:
        return q, k, v, D
    return (TF.pad(q, (0, Dp - D)), TF.pad(k, (0, Dp - D)), TF.pad(v, (0, Dp - D)), D)


def _hip_ok(q, k, v):
    if not ops.use_hip(q):
        return False
    D = q.shape[-1]
    Dp = ops.flash_attn.tiled_head_dim(D)
    # shape/dtype contract of the kernels, checked on the (padded) operand geometry
    return (q.dtype in (torch.bfloat16, torch.float16) and k.dtype == q.dtype and v.dtype == q.dtype
            and Dp is not None and k.shape[-1] == D and v.shape[-1] == D and k.shape == v.shape
            and k.shape[-2] > 0 and q.shape[-2] % k.shape[-2] == 0)


def _kernel_attend(q, k, v, causal, scale, mask=None, dropout=0.0, cu_q=None, cu_k=None, max_q=None, max_k=None,
                   start_rows=None):
    """HIP flash attention on BSHD (or packed varlen [total, H, D]) with optional mask /
    dropout / flashmask rows; pads unsupported head dims."""
    q, k, v, D = _pad_head(q, k, v)
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if not ops.flash_attn.supported(*(t.unsqueeze(0) if t.dim() == 3 else t for t in (q, k, v))):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
    plain = mask is None and dropout == 0.0 and cu_q is None and start_rows is None
    if plain:
        out = ops.flash_attn.flash_attention(q, k, v, causal, scale)
    else:
        out = ops.flash_attn.flash_attention_ex(q, k, v, causal, scale, mask, dropout, cu_q, cu_k, max_q, max_k,
                                                start_rows)
    return out if out.shape[-1] == D else out[..., :D]


def _attend(q, k, v, mask=None, dropout=0.0, causal=False, training=True, scale=None):
    if not training:
        dropout = 0.0
    if _hip_ok(q, k, v) and (mask is None or mask.dim() <= 4):
        return _kernel_attend(q, k, v, causal, scale, mask, dropout)
    return _sdpa_reference(q, k, v, mask, dropout, causal, scale)


@_amp_op('flash_attn')
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
    p = dropout if training else 0.0
    if t.dim() == 5 and t.shape[2] == 3 and not return_softmax and ops.use_hip(t) and ops.flash_attn.supported(q, k, v):
        # one packed gradient for the fused QKV projection (no per-view grad fill / copies)
        if p == 0.0:
            return _w(ops.flash_attn.flash_attention_packed(t, causal)), None
        return _w(ops.flash_attn.flash_attention_packed_ex(t, causal, dropout=p)), None
    return flash_attention(_w(q), _w(k), _w(v), dropout, causal, return_softmax, training=training)


def _unpadded_reference(q, k, v, cq, ck, scale, dropout, causal, training):
    cq, ck = cq.tolist(), ck.tolist()
    out = torch.zeros(q.shape[0], q.shape[1], v.shape[-1], dtype=q.dtype, device=q.device)
    for i in range(len(cq) - 1):
        qi = q[cq[i]:cq[i + 1]].unsqueeze(0)
        ki = k[ck[i]:ck[i + 1]].unsqueeze(0)
        vi = v[ck[i]:ck[i + 1]].unsqueeze(0)
        out[cq[i]:cq[i + 1]] = _sdpa_reference(qi, ki, vi, None, dropout if training else 0.0, causal, scale)[0]
    return out


def flash_attn_unpadded(query, key, value, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale,
                        dropout=0.0, causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                        training=True, name=None):
    """Variable-length attention over packed [total_tokens, heads, dim] tensors: one kernel
    launch over every sequence (grid over the longest; per-sequence bounds from cu_seqlens)."""
    q, k, v = _u(query), _u(key), _u(value)
    cq, ck = _u(cu_seqlens_q), _u(cu_seqlens_k)
    if _hip_ok(q, k, v) and not return_softmax:
        return _w(_kernel_attend(q, k, v, causal, scale, None, dropout if training else 0.0, cq, ck,
                                 int(max_seqlen_q), int(max_seqlen_k))), None
    return _w(_unpadded_reference(q, k, v, cq, ck, scale, dropout, causal, training)), None


def flash_attn_varlen_qkvpacked(qkv, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale, dropout=0.0,
                                causal=False, return_softmax=False, fixed_seed_offset=None, rng_name="",
                                varlen_padded=True, training=True, name=None):
    """qkv [total, nheads/nheads_k + 2, nheads_k, d] (reference flash_attention.py:594); rows
    outside every cu_seqlens span (the padding of a padded layout) come back as zeros."""
    t = _u(qkv)
    q = t[:, :-2].reshape(t.shape[0], -1, t.shape[-1])
    return flash_attn_unpadded(_w(q), _w(t[:, -2]), _w(t[:, -1]), cu_seqlens_q, cu_seqlens_k, max_seqlen_q,
                               max_seqlen_k, scale, dropout, causal, return_softmax, training=training)


@_amp_op('flash_attn')
def scaled_dot_product_attention(query, key, value, attn_mask=None, dropout_p=0.0, is_causal=False, training=True,
                                 name=None):
    q, k, v = _u(query), _u(key), _u(value)
    m = _u(attn_mask) if attn_mask is not None else None
    return _w(_attend(q, k, v, m, dropout_p, is_causal, training))


def flash_attention_with_sparse_mask(query, key, value, attn_mask_start_row_indices, attn_mask_start_row=0,
                                     dropout_p=0.0, is_causal=False, return_softmax=False, return_softmax_lse=False,
                                     return_seed_offset=False, training=True, name=None):
    """flashmask: key column k is masked for query rows >= attn_mask_start_row_indices[b, h, k]
    (reference flash_attention.py:844); on HIP the kernel reads the O(S) index vector directly."""
    q, k, v = _u(query), _u(key), _u(value)
    rows = _u(attn_mask_start_row_indices)  # [b, h, S_k]
    p = dropout_p if training else 0.0
    if _hip_ok(q, k, v):
        out = _kernel_attend(q, k, v, is_causal, None, None, p, start_rows=rows)
    else:
        S = q.shape[1]
        r = torch.arange(S, device=q.device).view(1, 1, S, 1)
        mask = r < rows.unsqueeze(2)
        if is_causal:
            mask = mask & torch.ones(S, k.shape[1], dtype=torch.bool, device=q.device).tril(k.shape[1] - S)
        out = _sdpa_reference(q, k, v, mask, p, False)
    return _w(out)


def sparse_attention(query, key, value, sparse_csr_offset, sparse_csr_columns, key_padding_mask=None, attn_mask=None,
                     name=None):
    """Attention restricted to a CSR sparsity pattern per (batch, head) (reference:
    python/paddle/nn/functional/sparse_attention.py): row i of (b, h) attends to the key columns
    ``sparse_csr_columns[b, h, offset[b, h, i]:offset[b, h, i + 1]]``.  ``key_padding_mask``
    ([batch, seq]) and ``attn_mask`` ([seq, seq]) zero entries mask positions out as well.
    The CSR pattern is expanded to a dense boolean mask on the device in one scatter (row of every
    stored entry by a batched searchsorted over the offsets) — no host loop."""
    q, k, v = _u(query), _u(key), _u(value)  # [b, h, s, d]
    off, cols = _u(sparse_csr_offset).long(), _u(sparse_csr_columns).long()
    B, H, S, D = q.shape
    Sk = k.shape[2]
    nnz = cols.shape[-1]
    idx = torch.arange(nnz, device=q.device).expand(B, H, nnz).contiguous()
    rows = torch.searchsorted(off[..., 1:].contiguous(), idx, right=True)  # row of every stored entry
    valid = idx < off[..., -1:]
    bi = torch.arange(B, device=q.device).view(B, 1, 1).expand(B, H, nnz)
    hi = torch.arange(H, device=q.device).view(1, H, 1).expand(B, H, nnz)
    mask = torch.zeros(B, H, S, Sk, dtype=torch.bool, device=q.device)
    mask[bi[valid], hi[valid], rows.clamp_max(S - 1)[valid], cols[valid]] = True
    if key_padding_mask is not None:
        mask &= (_u(key_padding_mask) != 0).view(B, 1, 1, Sk)
    if attn_mask is not None:
        mask &= (_u(attn_mask) != 0).view(1, 1, S, Sk)
    return _w(TF.scaled_dot_product_attention(q, k, v, attn_mask=mask))


def memory_efficient_attention(query, key, value, attn_bias=None, p=0.0, scale=None, training=True):
    q, k, v = _u(query), _u(key), _u(value)
    return _w(_attend(q, k, v, _u(attn_bias) if attn_bias is not None else None, p, False, training, scale))
