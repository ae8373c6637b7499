"""paddle.incubate.nn.functional fused ops (reference: python/paddle/incubate/nn/functional/*.py).

Each maps onto one hand-written HIP kernel on GPU tensors (csrc/*.hip) and onto an exact
composite of storage-layer ops on CPU.
"""
import math

import torch
import torch.nn.functional as TF

from ...core.tensor import Tensor, _wrap as _w, _unwrap as _u
from ... import ops
from ...nn import functional as F
from ...nn.functional.flash_attention import _attend
from ...core.amp_dispatch import amp_op as _amp_op


def fused_rms_norm(x, norm_weight, norm_bias=None, epsilon=1e-6, begin_norm_axis=-1, bias=None, residual=None,
                   quant_scale=-1, quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    """Returns (out, residual_out) like the reference (residual_out is x (+bias) + residual)."""
    t, w = _u(x), _u(norm_weight)
    if bias is not None:
        t = t + _u(bias)
    r = _u(residual) if residual is not None else None
    if ops.use_hip(t):
        if r is not None:
            y, s = ops.norm.add_rms_norm(t, r, w, epsilon)
        else:
            y, s = ops.norm.rms_norm(t, w, epsilon), t
    else:
        s = t + r if r is not None else t
        var = s.float().pow(2).mean(-1, keepdim=True)
        y = (s.float() * torch.rsqrt(var + epsilon)).to(s.dtype) * w.to(s.dtype)
    if norm_bias is not None:
        y = y + _u(norm_bias)
    return (_w(y), _w(s)) if residual is not None else _w(y)


def fused_layer_norm(x, norm_weight, norm_bias, epsilon, residual_alpha=1.0, begin_norm_axis=-1, bias=None,
                     residual=None, quant_scale=-1, quant_round_type=0, quant_max_bound=0, quant_min_bound=0):
    t, w = _u(x), _u(norm_weight)
    b = _u(norm_bias) if norm_bias is not None else None
    if bias is not None:
        t = t + _u(bias)
    r = _u(residual) if residual is not None else None
    if r is not None and residual_alpha != 1.0:
        r = r * residual_alpha
    if ops.use_hip(t) and b is not None:
        if r is not None:
            y, s = ops.norm.add_layer_norm(t, r, w, b, epsilon)
        else:
            y, s = ops.norm.layer_norm(t, w, b, epsilon), t
    else:
        s = t + r if r is not None else t
        y = TF.layer_norm(s, [s.shape[-1]], w.to(s.dtype) if w is not None else None,
                          b.to(s.dtype) if b is not None else None, epsilon)
    return (_w(y), _w(s)) if residual is not None else _w(y)


def fused_dropout_add(x, y, p=0.5, training=True, mode='upscale_in_train', name=None):
    t, r = _u(x), _u(y)
    if not training or p == 0.0:
        return _w(t + r)
    if ops.use_hip(t) and mode == 'upscale_in_train' and t.shape == r.shape:
        return _w(ops.act.dropout_add(t, r, p))
    return _w(TF.dropout(t, p, True) + r)


def fused_bias_dropout_residual_layer_norm(x, residual, bias=None, ln_scale=None, ln_bias=None, dropout_rate=0.5,
                                           ln_epsilon=1e-5, training=True, mode='upscale_in_train', name=None):
    """y = layer_norm(residual + dropout(x + bias)) (reference incubate/nn/functional/
    fused_transformer.py fused_bias_dropout_residual_layer_norm).  On the GPU one csrc/norm.hip
    kernel each way (keep mask regenerated from its counter hash in the backward)."""
    if mode not in ('upscale_in_train', 'downscale_in_infer'):
        raise ValueError("mode must be 'upscale_in_train' or 'downscale_in_infer'")
    t, r = _u(x), _u(residual)
    p = float(dropout_rate) if training else 0.0
    w = _u(ln_scale) if ln_scale is not None else None
    b = _u(ln_bias) if ln_bias is not None else None
    if (mode == 'upscale_in_train' and ops.use_hip(t) and w is not None and t.shape == r.shape
            and (bias is None or _u(bias).dtype == t.dtype) and ops.fused.dropout_add_norm_ok(t, w, p)):
        y, _ = ops.fused.dropout_add_norm(t, bias, r, w, b, float(ln_epsilon), p)
        return _w(y)
    h = t + _u(bias) if bias is not None else t
    if p > 0.0:
        h = TF.dropout(h, p, True)
    elif mode == 'downscale_in_infer' and dropout_rate > 0.0 and not training:
        h = h * (1.0 - dropout_rate)
    h = h + r
    y = TF.layer_norm(h.float(), [h.shape[-1]], w.float() if w is not None else None,
                      b.float() if b is not None else None, ln_epsilon).to(h.dtype)
    return _w(y)


@_amp_op('fused_rotary_position_embedding')
def fused_rotary_position_embedding(q, k=None, v=None, sin=None, cos=None, position_ids=None,
                                    use_neox_rotary_style=True, time_major=False, rotary_emb_base=10000.0):
    """q/k/v: [B, S, H, D].  use_neox_rotary_style=True rotates adjacent pairs (reference docstring)."""
    outs = []
    for x in (q, k, v):
        if x is None:
            outs.append(None)
            continue
        t = _u(x)
        if time_major:
            t = t.transpose(0, 1)
        B, S, H, D = t.shape
        if sin is not None and cos is not None:
            c = _u(cos).reshape(-1, _u(cos).shape[-1])[:, :D].float()
            s = _u(sin).reshape(-1, _u(sin).shape[-1])[:, :D].float()
            # reference passes full-D tables with duplicated halves/pairs; take the unique half
            if use_neox_rotary_style:
                c, s = c[:, 0::2].contiguous(), s[:, 0::2].contiguous()
            else:
                c, s = c[:, :D // 2].contiguous(), s[:, :D // 2].contiguous()
        else:
            c, s = ops.rope.rope_tables(max(S, 1) if position_ids is None else int(_u(position_ids).max()) + 1, D,
                                        rotary_emb_base, t.device)
        pos = _u(position_ids) if position_ids is not None else None
        if ops.use_hip(t):
            y = ops.rope.apply_rope(t, c, s, pos, interleaved=use_neox_rotary_style)
        else:
            y = _rope_ref(t, c, s, pos, use_neox_rotary_style)
        if time_major:
            y = y.transpose(0, 1)
        outs.append(_w(y))
    return tuple(outs)


def _rope_ref(t, c, s, pos, interleaved):
    B, S, H, D = t.shape
    if pos is None:
        cc, ss = c[:S][None, :, None, :], s[:S][None, :, None, :]
    else:
        cc, ss = c[pos][:, :, None, :], s[pos][:, :, None, :]
    tf = t.float()
    if interleaved:
        a, b = tf[..., 0::2], tf[..., 1::2]
        ra, rb = a * cc - b * ss, b * cc + a * ss
        return torch.stack([ra, rb], -1).flatten(-2).to(t.dtype)
    a, b = tf[..., :D // 2], tf[..., D // 2:]
    return torch.cat([a * cc - b * ss, b * cc + a * ss], -1).to(t.dtype)


def swiglu(x, y=None, name=None):
    return F.swiglu(x, y)


def fused_matmul_bias(x, y, bias=None, transpose_x=False, transpose_y=False, name=None):
    a, b = _u(x), _u(y)
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    if bias is not None and a.dim() == 2 and b.dim() == 2:
        return _w(ops.matmul.linear(a, b, _u(bias)))  # bias in the GEMM epilogue
    out = ops.matmul.matmul(a, b)
    return _w(out + _u(bias) if bias is not None else out)


def fused_linear(x, weight, bias=None, transpose_weight=False, name=None):
    return fused_matmul_bias(x, weight, bias, False, transpose_weight)


def fused_linear_activation(x, y, bias, trans_x=False, trans_y=False, activation=None):
    out = fused_matmul_bias(x, y, bias, trans_x, trans_y)
    if activation in (None, 'none', 'identity'):
        return out
    return getattr(F, activation)(out)


def fused_bias_act(x, bias=None, dequant_scales=None, shift=None, smooth=None, act_method='gelu',
                   compute_dtype='default', quant_scale=-1, quant_round_type=0, quant_max_bound=0,
                   quant_min_bound=0):
    t = _u(x)
    b = _u(bias) if bias is not None else None
    if act_method in ('swiglu', 'geglu'):
        t = t + b if b is not None else t
        a, g = t.chunk(2, -1)
        return _w(TF.silu(a) * g if act_method == 'swiglu' else TF.gelu(a) * g)
    if ops.use_hip(t):
        fn = {'gelu': ops.act.gelu, 'silu': ops.act.silu, 'relu': ops.act.bias_relu}[act_method]
        return _w(fn(t, bias=b))
    t = t + b if b is not None else t
    return _w({'gelu': TF.gelu, 'silu': TF.silu, 'relu': torch.relu}[act_method](t))


def _tp_in(h, g):
    from ...distributed.fleet.layers.mpu.mp_ops import _c_identity
    return _c_identity(h, group=g)  # identity forward, gradient all-reduced backward


def _tp_out(o, bias, g):
    from ...distributed.fleet.layers.mpu.mp_ops import _mp_allreduce
    o = _mp_allreduce(o, group=g)
    return o + bias if bias is not None else o


def fused_feedforward(x, linear1_weight, linear2_weight, linear1_bias=None, linear2_bias=None, ln1_scale=None,
                      ln1_bias=None, ln2_scale=None, ln2_bias=None, dropout1_rate=0.5, dropout2_rate=0.5,
                      activation="relu", ln1_epsilon=1e-5, ln2_epsilon=1e-5, pre_layer_norm=False, training=True,
                      mode='upscale_in_train', ring_id=-1, add_residual=True, name=None):
    """ring_id != -1: tensor parallel over that group — linear1 column-parallel (this rank's
    columns), linear2 row-parallel (its rows; the partial outputs all-reduced before the bias)."""
    residual = x
    h = x
    if pre_layer_norm:
        h = F.layer_norm(h, [_u(x).shape[-1]], ln1_scale, ln1_bias, ln1_epsilon)
    g = _ring_group(ring_id) if ring_id != -1 else None
    if g is not None:
        h = _tp_in(h, g)
    h = F.linear(h, linear1_weight, linear1_bias)
    h = getattr(F, activation)(h)
    h = F.dropout(h, dropout1_rate, training=training, mode=mode)
    h = F.linear(h, linear2_weight, linear2_bias) if g is None else _tp_out(F.linear(h, linear2_weight), linear2_bias, g)
    if add_residual:
        h = fused_dropout_add(h, residual, dropout2_rate, training, mode)
    else:
        h = F.dropout(h, dropout2_rate, training=training, mode=mode)
    if not pre_layer_norm:
        h = F.layer_norm(h, [_u(x).shape[-1]], ln2_scale, ln2_bias, ln2_epsilon)
    return h


def fused_multi_head_attention(x, qkv_weight, linear_weight, pre_layer_norm=False, pre_ln_scale=None,
                               pre_ln_bias=None, ln_scale=None, ln_bias=None, pre_ln_epsilon=1e-05, qkv_bias=None,
                               linear_bias=None, cache_kv=None, attn_mask=None, dropout_rate=0.5,
                               attn_dropout_rate=0.5, ln_epsilon=1e-05, training=True, mode='upscale_in_train',
                               ring_id=-1, add_residual=True, num_heads=-1, transpose_qkv_wb=False, name=None):
    """qkv_weight: [3, H, D, E] (reference layout) or [E, 3E] with transpose_qkv_wb=True.
    ring_id != -1: tensor parallel over that group — this rank's heads of qkv_weight / qkv_bias
    and rows of linear_weight; the out-linear partials are all-reduced before linear_bias."""
    t = _u(x)
    B, S, E = t.shape
    h = x
    if pre_layer_norm:
        h = F.layer_norm(h, [E], pre_ln_scale, pre_ln_bias, pre_ln_epsilon)
    g = _ring_group(ring_id) if ring_id != -1 else None
    if g is not None:
        h = _tp_in(h, g)  # with transpose_qkv_wb, num_heads is this rank's head count
    w = _u(qkv_weight)
    if transpose_qkv_wb:
        qkv = ops.matmul.matmul(_u(h), w)
        if qkv_bias is not None:
            qkv = qkv + _u(qkv_bias)
        H = num_heads
        qkv = qkv.reshape(B, S, 3, H, qkv.shape[-1] // (3 * H))
    else:
        _, H, D, _ = w.shape
        qkv = torch.einsum('bse,thde->bsthd', _u(h), w)
        if qkv_bias is not None:
            qkv = qkv + _u(qkv_bias).reshape(1, 1, 3, H, D)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o = F.scaled_dot_product_attention(_w(q), _w(k), _w(v), attn_mask, attn_dropout_rate, False, training)
    o = _w(_u(o).reshape(B, S, -1))
    o = F.linear(o, linear_weight, linear_bias) if g is None else _tp_out(F.linear(o, linear_weight), linear_bias, g)
    if add_residual:
        o = fused_dropout_add(o, x, dropout_rate, training, mode)
    if not pre_layer_norm:
        o = F.layer_norm(o, [E], ln_scale, ln_bias, ln_epsilon)
    return o


def _rope_rows(t, cos, sin, neox):
    """Rotary embedding on rows t [..., D] with per-row cos/sin [..., D] (full width)."""
    tf = t.float()
    if neox:
        h = tf.shape[-1] // 2
        rot = torch.cat([-tf[..., h:], tf[..., :h]], -1)
    else:
        rot = torch.stack([-tf[..., 1::2], tf[..., 0::2]], -1).reshape(tf.shape)
    return (tf * cos + rot * sin).to(t.dtype)


def _full_width(cs, D, neox):
    """cos/sin given for D/2 frequencies -> D columns in the layout of the rotation."""
    if cs.shape[-1] == D:
        return cs
    return torch.cat([cs, cs], -1) if neox else cs.repeat_interleave(2, -1)


def _quant_out(o, out_scale, out_shift, out_smooth, round_type, max_bound, min_bound):
    """int8 output quantisation of the fused inference kernels: ((o + shift) * smooth) scaled by
    max_bound * out_scale, rounded (type 0: half to even, 1: half away from zero) and clipped."""
    f = o.float()
    if out_shift is not None:
        f = f + _u(out_shift).float().reshape(1, -1)
    if out_smooth is not None:
        f = f * _u(out_smooth).float().reshape(1, -1)
    v = f * (max_bound * out_scale)
    v = torch.round(v) if round_type == 0 else torch.sign(v) * torch.floor(v.abs() + 0.5)
    return v.clamp(min_bound, max_bound).to(torch.int8)


def _compute_dtype(compute_dtype, *likes):
    m = {'bf16': torch.bfloat16, 'fp16': torch.float16, 'fp32': torch.float32}
    if compute_dtype in m:
        return m[compute_dtype]
    for t in likes:
        if t is not None and t.is_floating_point():
            return t.dtype
    return torch.float32


def _beam_gather(cache, beam_off, B, L):
    """Per-(beam, position) source rows: row b = bi * beam + j reads position p from row
    bi * beam + beam_off[bi, j, p] (the cache of the beam it descends from)."""
    nb = _u(beam_off).shape[1]
    base = (torch.arange(B, device=cache.device) // nb * nb)[:, None]
    src = base + _u(beam_off).reshape(B, -1)[:, :L].long()                        # [B, L]
    pos = torch.arange(L, device=cache.device)[None, :].expand(B, L)
    k = cache[0].permute(0, 2, 1, 3)[src, pos].permute(0, 2, 1, 3).contiguous()  # [B, H, L, D]
    v = cache[1].permute(0, 2, 1, 3)[src, pos].permute(0, 2, 1, 3).contiguous()
    return k, v


def masked_multihead_attention(x, cache_kv=None, bias=None, src_mask=None, cum_offsets=None, sequence_lengths=None,
                               rotary_tensor=None, beam_cache_offset=None, qkv_out_scale=None, out_shift=None,
                               out_smooth=None, seq_len=1, rotary_emb_dims=0, use_neox_rotary_style=False,
                               compute_dtype='default', out_scale=-1, quant_round_type=1, quant_max_bound=127.0,
                               quant_min_bound=-127.0):
    """One decode step of attention (reference incubate/nn/functional/masked_multihead_attention.py:19).

    x: [B, 3*H*D] fused qkv of the new token; cache_kv: [2, B, H, max_len, D] (updated IN PLACE:
    the new K/V land at step t = sequence_lengths[b] (or src_mask.shape[-1] - 1), then the token
    attends over positions [0, t]).  bias [3, H, D], src_mask additive [B, 1, 1, >= t+1],
    rotary_tensor [2, B, 1|seq, ..., D] (cos, sin).  Returns (out [B, H*D], cache_kv).  The
    attention runs on the split-K HIP decode kernel (csrc/decode_attn.hip); the cache layout is
    the natural [B, H, L, D] (the reference's CUDA kernel keeps K as [B, H, D/8, L, 8]).

    Quantised serving paths: ``qkv_out_scale`` [3, H, D] dequantises an int32 ``x`` (the int8 QKV
    GEMM's accumulator); ``out_scale > 0`` quantises the output to int8 after ``out_shift`` /
    ``out_smooth`` (round type and bounds as the reference).  Beam search: ``beam_cache_offset``
    [B / beam, beam, L] names, per beam and past position, the beam whose cache row holds that
    position; the call then returns (out, cache_kv, beam_cache_offset)."""
    t = _u(x)
    cache = _u(cache_kv)
    _, B, H, L, D = cache.shape
    if qkv_out_scale is not None:  # int32 accumulator -> real values
        t = (t.float() * _u(qkv_out_scale).float().reshape(1, -1)).to(_compute_dtype(compute_dtype, cache))
    qkv = t.reshape(B, 3, H, D)
    if sequence_lengths is not None:
        step = _u(sequence_lengths).reshape(-1).to(torch.int32)
    elif src_mask is not None:
        step = torch.full((B,), _u(src_mask).shape[-1] - 1, dtype=torch.int32, device=t.device)
    else:
        raise ValueError("masked_multihead_attention needs sequence_lengths or src_mask to know the decode step")
    bq = bk = bv = None
    if bias is not None:
        bb = _u(bias).reshape(3, H * D)
        bq, bk, bv = bb[0], bb[1], bb[2]
    q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
    if rotary_tensor is not None and rotary_emb_dims > 0:
        rt = _u(rotary_tensor).float()
        rt = rt.reshape(2, B, -1, rt.shape[-1])
        idx = (step.long().clamp_min(0) if rt.shape[2] > 1 else torch.zeros(B, dtype=torch.long, device=t.device))
        cos = _full_width(rt[0, torch.arange(B, device=t.device), idx], D, use_neox_rotary_style)[:, None]
        sin = _full_width(rt[1, torch.arange(B, device=t.device), idx], D, use_neox_rotary_style)[:, None]
        if bq is not None:
            q, k = q + bq.reshape(1, H, D), k + bk.reshape(1, H, D)
            bq = bk = None
        q = _rope_rows(q, cos, sin, use_neox_rotary_style)
        k = _rope_rows(k, cos, sin, use_neox_rotary_style)
    ops.decode.kv_cache_write(k, v, cache[0], cache[1], step, k_bias=bk, v_bias=bv)
    lens = torch.where(step >= 0, step + 1, torch.zeros_like(step))
    mask = None
    if src_mask is not None:
        mask = _u(src_mask).reshape(B, -1).float()
    if beam_cache_offset is not None:
        Lu = int(lens.max())
        kg, vg = _beam_gather(cache, beam_cache_offset, B, Lu)
        cur = step.long().clamp_min(0)  # the new token's K/V live in its own row
        ar = torch.arange(B, device=t.device)
        kg[ar, :, cur] = cache[0][ar, :, cur]
        vg[ar, :, cur] = cache[1][ar, :, cur]
        o = ops.decode.decode_attention(q, kg, vg, lens, mask=mask, q_bias=bq)
    else:
        o = ops.decode.decode_attention(q, cache[0], cache[1], lens, mask=mask, q_bias=bq)
    o = o.reshape(B, H * D)
    if out_scale > 0:
        o = _quant_out(o, out_scale, out_shift, out_smooth, quant_round_type, quant_max_bound, quant_min_bound)
    if beam_cache_offset is not None:
        return _w(o), _w(cache), beam_cache_offset
    return _w(o), _w(cache)


def block_multihead_attention(qkv, key_cache, value_cache, seq_lens_encoder, seq_lens_decoder, seq_lens_this_time,
                              padding_offsets, cum_offsets, cu_seqlens_q, cu_seqlens_k, block_tables,
                              pre_key_cache=None, pre_value_cache=None, cache_k_quant_scales=None,
                              cache_v_quant_scales=None, cache_k_dequant_scales=None, cache_v_dequant_scales=None,
                              qkv_out_scale=None, qkv_bias=None, out_shift=None, out_smooth=None,
                              max_enc_len_this_time=None, max_dec_len_this_time=None, rope_emb=None, mask=None,
                              tgt_mask=None, max_seq_len=-1, block_size=64, use_neox_style=False,
                              use_dynamic_cachekv_quant=False, quant_round_type=1, quant_max_bound=127.0,
                              quant_min_bound=-127.0, out_scale=-1, compute_dtype="default"):
    """Paged-KV-cache attention over a mixed batch (reference incubate/nn/functional/
    block_multihead_attention.py:19): sequences with seq_lens_encoder > 0 are prompts (all their
    tokens' K/V written into their cache blocks, causal attention over the prompt), the others
    decode one token at position seq_lens_decoder[b] over their cached prefix (split-K HIP decode
    kernel over the block table).  qkv: [token_num, (Hq + 2 Hkv) * D] unpadded;
    key_cache / value_cache: [num_blocks, Hkv, block_size, D] (updated in place).
    Returns (out [token_num, Hq*D], qkv, key_cache, value_cache).

    ``pre_key_cache`` / ``pre_value_cache`` [B, Hkv, P, D]: a per-sequence prefix every query
    attends to ahead of its own keys (prompts: before the causal prompt block; decode: before the
    paged prefix).  Static int8 KV caches: with ``cache_k_quant_scales`` / ``cache_v_quant_scales``
    ([Hkv]) the new K/V are stored as clip(round(x * quant_scale)) in int8 caches and read back as
    q * dequant_scale (``cache_*_dequant_scales``); the decode rows read the 8-bit pages directly
    and dequantise inside the HIP decode kernel (a dequantised copy only with pre-caches).  A uint8
    cache stores the value offset by 128 (the reference's layout), an int8 cache stores it as is.  ``use_dynamic_cachekv_quant``: the scales
    are [B, Hkv] and written here — every prompt sequence of the call gets quant scale
    max_bound / absmax (per head, over all the call's new K resp. V rows, as the reference's
    quant_write_cache_int8_kernel does) and dequant scale absmax / max_bound; decode rows
    quantise and dequantise with their sequence's stored scales."""
    t = _u(qkv)
    kc, vc = _u(key_cache), _u(value_cache)
    qcache = cache_k_quant_scales is not None
    if qcache and (cache_v_quant_scales is None or cache_k_dequant_scales is None or cache_v_dequant_scales is None):
        raise ValueError("int8 KV cache needs cache_{k,v}_quant_scales and cache_{k,v}_dequant_scales")
    if qkv_out_scale is not None:  # int32 QKV accumulator -> real values
        t = (t.float() * _u(qkv_out_scale).float().reshape(1, -1)).to(_compute_dtype(compute_dtype, kc))
    _, Hkv, bs, D = kc.shape
    T = t.shape[0]
    Hq = t.shape[1] // D - 2 * Hkv
    enc = _u(seq_lens_encoder).reshape(-1).to(torch.int32)
    dec = _u(seq_lens_decoder).reshape(-1).to(torch.int32)
    this = _u(seq_lens_this_time).reshape(-1).to(torch.int32)
    B = enc.shape[0]
    dev = t.device
    cu = _u(cu_seqlens_q).reshape(-1).to(torch.int64)
    bt = _u(block_tables).to(torch.int32)
    x = t + _u(qkv_bias).reshape(1, -1) if qkv_bias is not None else t
    q = x[:, :Hq * D].reshape(T, Hq, D)
    k = x[:, Hq * D:(Hq + Hkv) * D].reshape(T, Hkv, D)
    v = x[:, (Hq + Hkv) * D:].reshape(T, Hkv, D)
    # token -> (sequence, absolute position)
    seq_of = torch.repeat_interleave(torch.arange(B, device=dev, dtype=torch.int32), this.long(), output_size=T)
    start = cu[:-1][seq_of.long()]
    pos = (dec[seq_of.long()].long() + (torch.arange(T, device=dev) - start)).to(torch.int32)
    if rope_emb is not None:
        re = _u(rope_emb).float()                      # [2, B, max_seq, 1, D/2]
        cs = re.reshape(2, re.shape[1], re.shape[2], -1)
        cos = _full_width(cs[0, seq_of.long(), pos.long()], D, use_neox_style)[:, None]
        sin = _full_width(cs[1, seq_of.long(), pos.long()], D, use_neox_style)[:, None]
        q = _rope_rows(q, cos, sin, use_neox_style)
        k = _rope_rows(k, cos, sin, use_neox_style)
    if use_dynamic_cachekv_quant and not qcache:
        raise ValueError("use_dynamic_cachekv_quant needs the cache_{k,v}_(de)quant_scales tensors ([B, Hkv])")
    zero_pt = 128.0 if kc.dtype == torch.uint8 else 0.0
    if qcache:  # quantise the new rows into the int8 pages
        if use_dynamic_cachekv_quant:
            pre = (enc > 0)
            if bool(pre.any()):
                for x_, qs, dqs in ((k, cache_k_quant_scales, cache_k_dequant_scales),
                                    (v, cache_v_quant_scales, cache_v_dequant_scales)):
                    amax = x_.float().abs().amax(dim=(0, 2)).clamp_min(1e-30)          # [Hkv]
                    qv, dv = _u(qs).reshape(B, Hkv), _u(dqs).reshape(B, Hkv)
                    qv[pre] = (quant_max_bound / amax).to(qv.dtype)
                    dv[pre] = (amax / quant_max_bound).to(dv.dtype)

        ops.decode.kv_cache_write_q8(k, v, kc, vc, pos, _u(cache_k_quant_scales), _u(cache_v_quant_scales),
                                     seq_of=seq_of, block_tables=bt, round_type=quant_round_type,
                                     qmax=quant_max_bound, qmin=quant_min_bound)
    else:
        ops.decode.kv_cache_write(k, v, kc, vc, pos, seq_of=seq_of, block_tables=bt)
    out = torch.empty(T, Hq, D, dtype=t.dtype, device=dev)
    pre_k = _u(pre_key_cache) if pre_key_cache is not None else None
    pre_v = _u(pre_value_cache) if pre_value_cache is not None else None
    P = pre_k.shape[2] if pre_k is not None else 0
    enc_l, dec_b = enc.tolist(), ((enc == 0) & (this > 0)).nonzero().reshape(-1)
    # prompts: causal attention over the prompt's own tokens (flash kernel per prompt)
    for b, L in enumerate(enc_l):
        if L <= 0:
            continue
        s0 = int(cu[b])
        qb, kb, vb = q[s0:s0 + L][None], k[s0:s0 + L][None], v[s0:s0 + L][None]
        m = None if mask is None else _u(mask)[b:b + 1, :, :L, :L]
        if P:
            kb = torch.cat([pre_k[b].permute(1, 0, 2)[None].to(kb.dtype), kb], 1)
            vb = torch.cat([pre_v[b].permute(1, 0, 2)[None].to(vb.dtype), vb], 1)
            qi = torch.arange(L, device=dev)[:, None]
            ki = torch.arange(P + L, device=dev)[None, :]
            causal = torch.where(ki <= qi + P, 0.0, float('-inf')).to(torch.float32)[None, None]
            m = causal if m is None else torch.cat([torch.zeros(1, m.shape[1], L, P, device=dev), m.float()], -1)
            out[s0:s0 + L] = _attend(qb, kb, vb, m, 0.0, False, False)[0]
        else:
            out[s0:s0 + L] = _attend(qb, kb, vb, m, 0.0, m is None, False)[0]
    # decode tokens: one per sequence, over its paged prefix
    if dec_b.numel():
        rows = cu[:-1][dec_b.long()]
        lens = dec[dec_b.long()] + 1
        tm = None if tgt_mask is None else _u(tgt_mask).reshape(_u(tgt_mask).shape[0], -1)[dec_b.long()].float()
        if qcache and not P:
            # 8-bit pages dequantised inside the decode kernel (scales per KV head or per sequence)
            def dsc(sc):
                s_ = _u(sc).float()
                return s_.reshape(B, Hkv)[dec_b.long()] if use_dynamic_cachekv_quant else s_.reshape(Hkv)
            out[rows] = ops.decode.decode_attention(q[rows], kc, vc, lens, block_tables=bt[dec_b.long()], mask=tm,
                                                    k_dequant=dsc(cache_k_dequant_scales),
                                                    v_dequant=dsc(cache_v_dequant_scales))
        elif P or qcache:
            # contiguous copies of the decode rows' pages (dequantised), prefix keys in front
            nblk = bt.shape[1]
            pages = bt[dec_b.long()].long()                                   # [n, nblk]
            kd = kc[pages].permute(0, 2, 1, 3, 4).reshape(len(pages), Hkv, nblk * bs, D)
            vd = vc[pages].permute(0, 2, 1, 3, 4).reshape(len(pages), Hkv, nblk * bs, D)
            if qcache:
                def dqz(x_, sc):
                    s_ = _u(sc).float()
                    s_ = s_.reshape(B, Hkv)[dec_b.long()] if use_dynamic_cachekv_quant else s_.reshape(1, -1)
                    return ((x_.float() - zero_pt) * s_[:, :, None, None]).to(q.dtype)
                kd, vd = dqz(kd, cache_k_dequant_scales), dqz(vd, cache_v_dequant_scales)
            if P:
                kd = torch.cat([pre_k[dec_b.long()].to(kd.dtype), kd], 2)
                vd = torch.cat([pre_v[dec_b.long()].to(vd.dtype), vd], 2)
                if tm is not None:
                    tm = torch.cat([torch.zeros(tm.shape[0], P, device=dev), tm], 1)
            out[rows] = ops.decode.decode_attention(q[rows], kd.contiguous(), vd.contiguous(), lens + P, mask=tm)
        else:
            out[rows] = ops.decode.decode_attention(q[rows], kc, vc, lens, block_tables=bt[dec_b.long()], mask=tm)
    o = out.reshape(T, Hq * D)
    if out_scale > 0:
        o = _quant_out(o, out_scale, out_shift, out_smooth, quant_round_type, quant_max_bound, quant_min_bound)
    return _w(o), qkv, key_cache, value_cache


def _ring_group(ring_id):
    from ...distributed.communication import get_group
    g = get_group(ring_id) if ring_id else None
    if g is None:
        from ...distributed import fleet
        hcg = fleet.get_hybrid_communicate_group() if hasattr(fleet, 'get_hybrid_communicate_group') else None
        g = hcg.get_model_parallel_group() if hcg is not None else None
    if g is None:
        raise ValueError(f"ring_id {ring_id}: no such communication group (create it with "
                         "paddle.distributed.new_group or fleet.init)")
    return g


def fused_multi_transformer(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights, linear_biases,
                            ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases, ffn2_weights, ffn2_biases,
                            pre_layer_norm=True, epsilon=1e-05, residual_alpha=1.0, cache_kvs=None, beam_offset=None,
                            pre_caches=None, seq_lens=None, rotary_embs=None, time_step=None, attn_mask=None,
                            dropout_rate=0.0, rotary_emb_dims=0, activation="gelu", training=False,
                            mode='upscale_in_train', trans_qkvw=True, ring_id=-1, norm_type="layernorm",
                            use_neox_rotary_style=False, gqa_group_size=-1, name=None,
                            qkv_out_scales=None, out_linear_out_scales=None, ffn1_out_scales=None,
                            ffn2_out_scales=None, qkv_in_scale=None, out_linear_in_scale=None, ffn1_in_scale=None,
                            ffn2_in_scale=None, quant_round_type=1, quant_max_bound=127.0, quant_min_bound=-127.0):
    """A stack of transformer blocks in one call (reference incubate/nn/functional/
    fused_transformer.py:964).  Per layer: (pre-)norm -> fused QKV GEMM -> attention -> out proj
    -> residual -> (pre-)norm -> FFN1 -> activation -> FFN2 -> residual.

    * context / prefill (time_step None): causal flash attention over the sequence (attn_mask,
      if given, replaces the causal mask); with cache_kvs the K/V of every position are written
      into cache_kvs[i] ([2, B, Hkv, max_len, D]);
    * decode (time_step = t, x [B, 1, E]): the token's K/V are written at position t and it
      attends over [0, t] on the split-K HIP decode kernel (attn_mask: additive [B, 1, 1, t+1]).
    GEMMs go through ops.gemm.mm (hand-written MFMA kernel for large token counts), norms
    through the fused norm kernels.  Returns out, or (out, cache_kvs) when caches are given.

    ``pre_caches[i]`` ([2, B, Hkv, P, D], a shared prefix such as a system prompt) is attended to
    ahead of the sequence by every query (prefill and decode); ``beam_offset`` [B / beam, beam, L]
    selects, per beam and past position, the cache row of the beam it descends from (decode).

    Tensor parallelism (``ring_id`` != -1): the caller passes this rank's shard — qkv / ffn1 weights
    split by heads / columns, out-linear / ffn2 weights split by rows — and the partial outputs of
    the out-linear and ffn2 GEMMs are all-reduced over the group ``ring_id`` (a
    paddle.distributed group id; the fleet model-parallel group when no such group exists) before
    their (replicated) biases are added.

    Inside a captured decode step (``DecodeStepGraph``: a device ``time_step`` during capture)
    only ``time_step`` is re-read per replay as a value; ``attn_mask``, ``rotary_embs`` and
    ``seq_lens`` are graph inputs by ADDRESS — the replay reads whatever their storage holds, so
    they must be static buffers the caller refills in place (``buf.copy_(new)``) before each
    replay; a freshly allocated tensor per step would be silently ignored.

    int8 weights (``fused_multi_transformer_int8``, reference fused_multi_transformer_int8_op.cu):
    a Linear whose weight is int8 — laid out [out, in] (qkv [3, H, D, E] with trans_qkvw) — runs
    quantise (per-layer calibrated ``*_in_scale``) -> int8 GEMM -> dequantise by the per-channel
    ``*_out_scales`` [N] + bias on ops.int8.static_int8_linear (int8 MFMA GEMM / W8A16 decode
    kernel on the GPU)."""
    tp_group = _ring_group(ring_id) if ring_id != -1 else None
    qcfg = dict(round_type=quant_round_type, max_bound=quant_max_bound, min_bound=quant_min_bound)

    def qsc(ins, outs, i):
        if outs is None:
            return None
        if ins is None:
            raise ValueError("fused_multi_transformer: int8 weights need the *_in_scale of every Linear")
        return float(ins[i]), _u(outs[i])

    def row_parallel(t, w, b, q=None):
        o_ = lin(t, w, None, q=q)
        import torch.distributed as tdist
        tdist.all_reduce(o_, group=tp_group.pg)
        return o_ + _u(b).reshape(1, -1).to(o_.dtype) if b is not None else o_
    h = _u(x)
    B, S, E = h.shape
    nl = len(qkv_weights)
    # a device-resident time_step inside a hipGraph capture (DecodeStepGraph) stays on the device:
    # positions / lengths / the rotary row are derived from it there (no host read)
    ts_t = _u(time_step) if isinstance(time_step, Tensor) or torch.is_tensor(time_step) else None
    dev_step = ts_t is not None and ts_t.is_cuda and torch.cuda.is_current_stream_capturing()
    if dev_step:
        if beam_offset is not None or pre_caches is not None:
            raise ValueError("fused_multi_transformer: beam_offset / pre_caches need a host time_step "
                             "(not supported inside a captured decode step)")
        step = -1  # decode, position on the device
    else:
        step = None if time_step is None else int(ts_t.reshape(-1)[0]) if ts_t is not None else int(time_step)

    def norm(t, w, b):
        if norm_type == 'rmsnorm':
            return _u(fused_rms_norm(_w(t), w, b, epsilon))
        return _u(F.layer_norm(_w(t), [E], w, b, epsilon))

    def lin(t, w, b, trans=False, q=None, i8_kn=False):
        t2 = t.reshape(-1, t.shape[-1])
        wt = _u(w)
        if wt.dtype == torch.int8:  # [N, K] int8; i8_kn: the qkv weight [K, N] without trans_qkvw
            if q is None:
                raise ValueError("fused_multi_transformer: int8 weights need *_out_scales and *_in_scale")
            wq = wt.t() if i8_kn else wt
            return ops.int8.static_int8_linear(t2, wq.contiguous(), q[1], q[0],
                                               None if b is None else _u(b).reshape(-1), **qcfg)
        wt = wt.t() if trans else wt
        bb = None if b is None else _u(b).reshape(-1)
        if bb is not None and bb.dtype == t2.dtype and ops.gemm._skinny_wins(t2.shape[0], wt.shape[1], t2.shape[1]):
            return ops.gemm.mm(t2, wt, bias=bb)  # decode GEMM: the bias is added in its finishing pass
        y = ops.gemm.mm(t2, wt, bias=None)
        if bb is not None:
            y = y + bb.reshape(1, -1)
        return y

    # pre-LN with unit residual scale: every residual add is fused into the following norm kernel
    # (fused_layer_norm / fused_rms_norm with residual=), carried as (pending delta, stream)
    fuse_res = pre_layer_norm and residual_alpha == 1.0

    def norm_add(delta, stream, w, b):
        if norm_type == 'rmsnorm':
            y, s_ = fused_rms_norm(_w(delta), w, b, epsilon, residual=_w(stream))
        else:
            y, s_ = fused_layer_norm(_w(delta), w, b, epsilon, residual=_w(stream))
        return _u(y), _u(s_)

    def act(t):
        if activation == 'gelu':
            return TF.gelu(t)
        if activation == 'relu':
            return torch.relu(t)
        if activation == 'swiglu' and t.is_cuda:
            return _u(swiglu(_w(t)))  # one fused kernel over the two halves (no silu + mul pair)
        if activation in ('swiglu', 'geglu'):
            a, g = t.chunk(2, -1)
            return (TF.silu(a) if activation == 'swiglu' else TF.gelu(a)) * g
        raise ValueError(f"unsupported activation {activation}")

    caches_out = []
    pending = None  # fuse_res: the previous block's ffn2 output, not yet added to the stream h
    if dev_step:
        pos_step = ts_t.reshape(-1)[:1].to(torch.int32).expand(B).contiguous()
        lens_step = pos_step + 1
    elif step is not None:  # decode: one position per sequence, the same for every layer
        pos_step = torch.full((B,), step, dtype=torch.int32, device=h.device)
        lens_step = pos_step + 1
    for i in range(nl):
        if pending is not None:
            a, h = norm_add(pending, h, ln_scales[i], ln_biases[i] if ln_biases is not None else None)
            pending = None
        else:
            a = norm(h, ln_scales[i], ln_biases[i] if ln_biases is not None else None) if pre_layer_norm else h
        resid = h
        w = _u(qkv_weights[i])
        qb = qkv_biases[i] if qkv_biases is not None else None
        if trans_qkvw:
            Wm = w.reshape(-1, E)                                  # [(Hq + 2 Hkv) * D, E]
            qkv = lin(a, Wm, qb, trans=True, q=qsc(qkv_in_scale, qkv_out_scales, i))
        else:
            Wm = w.reshape(E, -1)
            qkv = lin(a, Wm, qb, q=qsc(qkv_in_scale, qkv_out_scales, i), i8_kn=True)
        if gqa_group_size > 0:
            D = w.shape[-2] if trans_qkvw else w.shape[-1]
            Hkv = gqa_group_size
            Hq = qkv.shape[-1] // D - 2 * Hkv
        else:
            D = w.shape[2] if trans_qkvw else w.shape[-1]
            Hq = Hkv = qkv.shape[-1] // (3 * D)
        qkv = qkv.reshape(B, S, Hq + 2 * Hkv, D)
        q, k, v = qkv[:, :, :Hq], qkv[:, :, Hq:Hq + Hkv], qkv[:, :, Hq + Hkv:]
        if rotary_embs is not None and rotary_emb_dims > 0:
            re = _u(rotary_embs).float().reshape(2, B, -1, D)      # [2, B, seq, D]
            if step is None:
                cos, sin = re[0][:, :S, None], re[1][:, :S, None]
            elif dev_step:
                idx = pos_step[:1].long().clamp_max(re.shape[2] - 1)
                cos, sin = re[0].index_select(1, idx)[:, :, None], re[1].index_select(1, idx)[:, :, None]
            else:
                idx = min(step, re.shape[2] - 1)
                cos, sin = re[0][:, idx:idx + 1, None], re[1][:, idx:idx + 1, None]
            q = _rope_rows(q, cos, sin, use_neox_rotary_style)
            k = _rope_rows(k, cos, sin, use_neox_rotary_style)
        cache = _u(cache_kvs[i]) if cache_kvs is not None else None
        if step is None:
            if cache is not None:  # prefill: every position's K/V into the cache
                pos = torch.arange(S, device=h.device, dtype=torch.int32).repeat(B)
                seq = torch.arange(B, device=h.device, dtype=torch.int32).repeat_interleave(S)
                if seq_lens is not None:
                    sl = _u(seq_lens).reshape(-1).to(torch.int32)
                    pos = torch.where(pos < sl.repeat_interleave(S), pos, torch.full_like(pos, -1))
                ops.decode.kv_cache_write(k.reshape(B * S, Hkv, D), v.reshape(B * S, Hkv, D), cache[0], cache[1],
                                          pos, seq_of=seq)
            m = _u(attn_mask) if attn_mask is not None else None
            if pre_caches is not None:  # prefix keys first: every query sees the whole prefix
                pc = _u(pre_caches[i])
                P = pc.shape[3]
                kk = torch.cat([pc[0].permute(0, 2, 1, 3).to(k.dtype), k], 1)
                vv = torch.cat([pc[1].permute(0, 2, 1, 3).to(v.dtype), v], 1)
                if m is None:
                    qi = torch.arange(S, device=h.device)[:, None]
                    ki = torch.arange(P + S, device=h.device)[None, :]
                    m = torch.where(ki <= qi + P, 0.0, float('-inf')).to(torch.float32)[None, None]
                o = _attend(q, kk, vv, m, 0.0, False, False)
            else:
                o = _attend(q, k, v, m, 0.0, m is None, False)
        else:
            if cache is None:
                raise ValueError("fused_multi_transformer decode (time_step) needs cache_kvs")
            pos = pos_step
            ops.decode.kv_cache_write(k[:, 0], v[:, 0], cache[0], cache[1], pos)
            lens = lens_step
            m = None if attn_mask is None else _u(attn_mask).reshape(B, -1).float()
            kc, vc = cache[0], cache[1]
            if beam_offset is not None:
                kc, vc = _beam_gather(cache, beam_offset, B, step + 1)
                ar = torch.arange(B, device=h.device)
                kc[ar, :, step], vc[ar, :, step] = cache[0][ar, :, step], cache[1][ar, :, step]
            if pre_caches is not None:
                pc = _u(pre_caches[i])
                kc = torch.cat([pc[0].to(kc.dtype), kc[:, :, :step + 1]], 2)
                vc = torch.cat([pc[1].to(vc.dtype), vc[:, :, :step + 1]], 2)
                lens = lens + pc.shape[3]
                if m is not None:
                    m = torch.cat([torch.zeros(B, pc.shape[3], device=m.device), m], 1)
            o = ops.decode.decode_attention(q[:, 0], kc.contiguous(), vc.contiguous(), lens, mask=m)[:, None]
        if cache is not None:
            caches_out.append(cache_kvs[i])
        o = (row_parallel if tp_group is not None else lin)(
            o.reshape(B, S, Hq * D), linear_weights[i], linear_biases[i] if linear_biases is not None else None,
            q=qsc(out_linear_in_scale, out_linear_out_scales, i))
        if fuse_res:
            f, h = norm_add(o.reshape(B, S, E).to(resid.dtype), resid, ffn_ln_scales[i],
                            ffn_ln_biases[i] if ffn_ln_biases is not None else None)
        else:
            h = resid * residual_alpha + o.reshape(B, S, E).to(resid.dtype)
            if not pre_layer_norm:
                h = norm(h, ln_scales[i], ln_biases[i] if ln_biases is not None else None)
            f = norm(h, ffn_ln_scales[i], ffn_ln_biases[i] if ffn_ln_biases is not None else None) \
                if pre_layer_norm else h
        resid = h
        f = act(lin(f, ffn1_weights[i], ffn1_biases[i] if ffn1_biases is not None else None,
                    q=qsc(ffn1_in_scale, ffn1_out_scales, i)))
        f = (row_parallel if tp_group is not None else lin)(
            f, ffn2_weights[i], ffn2_biases[i] if ffn2_biases is not None else None,
            q=qsc(ffn2_in_scale, ffn2_out_scales, i))
        if fuse_res:
            pending = f.reshape(B, S, E).to(resid.dtype)
            continue
        h = resid * residual_alpha + f.reshape(B, S, E).to(resid.dtype)
        if not pre_layer_norm:
            h = norm(h, ffn_ln_scales[i], ffn_ln_biases[i] if ffn_ln_biases is not None else None)
    if pending is not None:
        h = h + pending
    out = _w(h)
    return (out, caches_out) if cache_kvs is not None else out


def fused_multi_transformer_int8(x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights, linear_biases,
                                 ffn_ln_scales, ffn_ln_biases, ffn1_weights, ffn1_biases, ffn2_weights, ffn2_biases,
                                 pre_layer_norm=True, epsilon=1e-05, cache_kvs=None, time_step=None, attn_mask=None,
                                 dropout_rate=0.0, activation="gelu", training=False, mode='upscale_in_train',
                                 trans_qkvw=True, ring_id=-1, name=None, qkv_out_scales=None,
                                 out_linear_out_scales=None, ffn1_out_scales=None, ffn2_out_scales=None, num_head=0,
                                 dim_head=0, dim_ffn=0, qkv_in_scale=(), out_linear_in_scale=(), ffn1_in_scale=(),
                                 ffn2_in_scale=(), quant_round_type=1, quant_max_bound=127.0, quant_min_bound=-127.0):
    """The int8 FusedMultiTransformer (reference paddle/fluid/operators/fused/
    fused_multi_transformer_int8_op.cc; API as in test/legacy_test/test_fused_multi_transformer_int8_op.py:32):
    int8 weights [out, in] (qkv [3, H, D, E]), per-layer calibrated activation scales ``*_in_scale``
    (floats) and per-output-channel dequant scales ``*_out_scales`` ([N] fp32).  Every Linear runs
    quantise -> int8 GEMM -> dequantise + bias (ops.int8.static_int8_linear); norms, attention and
    the KV cache are the 16-bit fused_multi_transformer path.  num_head / dim_head / dim_ffn are
    implied by the weight shapes."""
    return fused_multi_transformer(
        x, ln_scales, ln_biases, qkv_weights, qkv_biases, linear_weights, linear_biases, ffn_ln_scales,
        ffn_ln_biases, ffn1_weights, ffn1_biases, ffn2_weights, ffn2_biases, pre_layer_norm=pre_layer_norm,
        epsilon=epsilon, cache_kvs=cache_kvs, time_step=time_step, attn_mask=attn_mask, dropout_rate=dropout_rate,
        activation=activation, training=training, mode=mode, trans_qkvw=trans_qkvw, ring_id=ring_id,
        qkv_out_scales=qkv_out_scales, out_linear_out_scales=out_linear_out_scales, ffn1_out_scales=ffn1_out_scales,
        ffn2_out_scales=ffn2_out_scales, qkv_in_scale=qkv_in_scale, out_linear_in_scale=out_linear_in_scale,
        ffn1_in_scale=ffn1_in_scale, ffn2_in_scale=ffn2_in_scale, quant_round_type=quant_round_type,
        quant_max_bound=quant_max_bound, quant_min_bound=quant_min_bound)


def variable_length_memory_efficient_attention(query, key, value, seq_lens, kv_seq_lens, mask=None, scale=None,
                                               causal=False, pre_cache_length=0):
    q, k, v = _u(query), _u(key), _u(value)  # [B, H, S, D]
    B, H, S, D = q.shape
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    s = torch.einsum('bhqd,bhkd->bhqk', q.float(), k.float()) * scale
    sl, kl = _u(seq_lens).reshape(-1), _u(kv_seq_lens).reshape(-1)
    qi = torch.arange(S, device=q.device)[None, None, :, None]
    ki = torch.arange(k.shape[2], device=q.device)[None, None, None, :]
    valid = (qi < sl.view(B, 1, 1, 1)) & (ki < kl.view(B, 1, 1, 1))
    if causal:
        valid = valid & (ki <= qi + pre_cache_length)
    if mask is not None:
        s = s + _u(mask).float()
    s = s.masked_fill(~valid, float('-inf'))
    p = torch.nan_to_num(torch.softmax(s, -1))
    return _w(torch.einsum('bhqk,bhkd->bhqd', p, v.float()).to(q.dtype))


def fused_dot_product_attention(q, k, v, mask, scaling_factor, dropout_prob, is_training, is_causal_masking,
                                use_workspace_opt=None, return_softmax=False):
    """Scaled dot-product attention on BSHD bf16 / fp16 (reference
    incubate/nn/functional/fused_dot_product_attention.py:22, a cuDNN fused kernel there): the
    hand-written flash-attention kernel (csrc/flash_attn.hip) with the int / bool keep-mask
    [B, 1, Sq, Sk] (1 = attend) or causal masking, in-kernel dropout and ``scaling_factor``.
    ``return_softmax`` additionally returns the [B, H, Sq, Sk] probabilities (recomputed)."""
    qt, kt, vt = _u(q), _u(k), _u(v)
    B, Sq, Sk = qt.shape[0], qt.shape[1], kt.shape[1]
    m = None
    if mask is not None and not is_causal_masking:
        mt = _u(mask)
        if tuple(mt.shape) != (B, 1, Sq, Sk):
            raise ValueError(f"mask shape must be [batch_size, 1, q_seqlen, k_seqlen], got {list(mt.shape)}")
        m = mt.bool() if mt.dtype != torch.bool else mt
        if bool(m.all()):
            m = None  # the reference's all-ones default
    p = float(dropout_prob) if is_training else 0.0
    out = _attend(qt, kt, vt, m, p, bool(is_causal_masking), bool(is_training), scale=float(scaling_factor))
    if not return_softmax:
        return _w(out)
    s = torch.einsum('bqhd,bkhd->bhqk', qt.float(), kt.float()) * float(scaling_factor)
    if is_causal_masking:
        s = s.masked_fill(torch.ones(Sq, Sk, dtype=torch.bool, device=s.device).tril(Sk - Sq).logical_not(),
                          float('-inf'))
    elif m is not None:
        s = s.masked_fill(~m, float('-inf'))
    return _w(out), _w(torch.softmax(s, -1).to(qt.dtype))


def fused_gate_attention(query, key=None, query_weight=None, key_weight=None, value_weight=None, qkv_weight=None,
                         gate_linear_weight=None, gate_linear_bias=None, out_linear_weight=None,
                         out_linear_bias=None, nonbatched_bias=None, attn_mask=None, has_gating=True,
                         merge_qkv=True, use_flash_attn=False):
    """AlphaFold-style gated self-attention over [batch, msa_len, res_len, q_dim] (reference
    incubate/nn/functional/fused_gate_attention.py:19):
      q, k, v = projections (packed qkv_weight [3, H, c, q_dim], or separate [dim, H, c] weights)
      logits  = q k^T * c^-0.5 + attn_mask [B, msa, 1, 1, m] (+ nonbatched_bias [B, 1, H, res, m])
      o       = softmax(logits) v  (* sigmoid(query @ gate_w + gate_b) when has_gating)
      out     = o @ out_linear_weight [H, c, q_dim] + out_linear_bias.
    Every projection and both attention products are two-operand contractions on the hand-written
    (batched) GEMM for bf16 / fp16 GPU operands (ops/matmul.py); the softmax runs in fp32."""
    qd = _u(query)
    if merge_qkv:
        if qkv_weight is None:
            raise ValueError("fused_gate_attention: merge_qkv=True needs qkv_weight [3, H, c, q_dim]")
        w = _u(qkv_weight)
        H, c = w.shape[1], w.shape[2]
        qkv = ops.matmul.matmul(qd.reshape(-1, qd.shape[-1]), w.reshape(3 * H * c, -1).t().to(qd.dtype))
        qkv = qkv.reshape(*qd.shape[:-1], 3, H, c)
        q, k, v = qkv[..., 0, :, :], qkv[..., 1, :, :], qkv[..., 2, :, :]
    else:
        md = _u(key) if key is not None else qd
        qw, kw, vw = _u(query_weight), _u(key_weight), _u(value_weight)
        H, c = qw.shape[1], qw.shape[2]
        q = ops.matmul.matmul(qd.reshape(-1, qd.shape[-1]), qw.reshape(qw.shape[0], -1).to(qd.dtype))
        k = ops.matmul.matmul(md.reshape(-1, md.shape[-1]), kw.reshape(kw.shape[0], -1).to(qd.dtype))
        v = ops.matmul.matmul(md.reshape(-1, md.shape[-1]), vw.reshape(vw.shape[0], -1).to(qd.dtype))
        q = q.reshape(*qd.shape[:-1], H, c)
        k = k.reshape(*md.shape[:-1], H, c)
        v = v.reshape(*md.shape[:-1], H, c)
    q = q * (c ** -0.5)
    # [n, b, q, h, c] -> [n, b, h, q, c]
    qh, kh, vh = q.permute(0, 1, 3, 2, 4), k.permute(0, 1, 3, 2, 4), v.permute(0, 1, 3, 2, 4)
    logits = ops.matmul.matmul(qh, kh.transpose(-1, -2)).float()          # [n, b, h, q, m]
    if attn_mask is not None:
        logits = logits + _u(attn_mask).float()
    if nonbatched_bias is not None:
        logits = logits + _u(nonbatched_bias).float()
    wts = torch.softmax(logits, -1).to(vh.dtype)
    o = ops.matmul.matmul(wts, vh).permute(0, 1, 3, 2, 4)                  # [n, b, q, h, c]
    if has_gating:
        gw, gb = _u(gate_linear_weight), _u(gate_linear_bias)
        gv = ops.matmul.matmul(qd.reshape(-1, qd.shape[-1]), gw.reshape(gw.shape[0], -1).to(qd.dtype))
        gv = gv.reshape(*qd.shape[:-1], H, c) + gb.to(gv.dtype)
        o = o * torch.sigmoid(gv.float()).to(o.dtype)
    ow = _u(out_linear_weight)
    out = ops.matmul.matmul(o.reshape(-1, H * c), ow.reshape(H * c, -1).to(o.dtype))
    if out_linear_bias is not None:
        out = out + _u(out_linear_bias).to(out.dtype)
    return _w(out.reshape(*qd.shape[:-1], -1))


def fused_ec_moe(x, gate, bmm0_weight, bmm0_bias, bmm1_weight, bmm1_bias, act_type):
    """Every token through every expert, combined with the softmaxed gate (reference
    incubate/nn/functional/fused_ec_moe.py:18, kernel fusion/cutlass/moe_kernel.cu).  The expert
    FFNs are two batched GEMMs over the experts (ops/matmul.py: the token matrix broadcast to every
    expert at batch stride 0, blockIdx.y = expert) — no per-expert loop, no weight copies."""
    t, g = _u(x), _u(gate)
    B, S, D = t.shape
    probs = torch.softmax(g.float(), -1)                       # [B, S, E]
    w0, w1 = _u(bmm0_weight), _u(bmm1_weight)                  # [E, D, F], [E, F, D]
    E = w0.shape[0]
    t2 = t.reshape(1, B * S, D)
    h = ops.matmul.matmul(t2, w0) + _u(bmm0_bias).reshape(E, 1, -1).to(t.dtype)   # [E, T, F]
    h = TF.gelu(h) if act_type == 'gelu' else torch.relu(h)
    o = ops.matmul.matmul(h, w1) + _u(bmm1_bias).reshape(E, 1, -1).to(t.dtype)    # [E, T, D]
    pr = probs.reshape(B * S, E).t().unsqueeze(-1).to(o.dtype)                     # [E, T, 1]
    return _w((o * pr).sum(0).reshape(B, S, D))


def blha_get_max_len(seq_lens_encoder, seq_lens_decoder, batch_size):
    return _w(_u(seq_lens_encoder).max().reshape(1)), _w(_u(seq_lens_decoder).max().reshape(1))
