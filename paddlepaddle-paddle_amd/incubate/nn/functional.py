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
    if bias is not None and a.dim() == 2:
        return _w(torch.addmm(_u(bias), a, b))
    out = torch.matmul(a, b)
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


def fused_feedforward(x, linear1_weight, linear2_weight, linear1_bias=None, linear2_bias=None, ln1_scale=None,
                      ln1_bias=None, ln2_scale=None, ln2_bias=None, dropout1_rate=0.5, dropout2_rate=0.5,
                      activation="relu", ln1_epsilon=1e-5, ln2_epsilon=1e-5, pre_layer_norm=False, training=True,
                      mode='upscale_in_train', ring_id=-1, add_residual=True, name=None):
    residual = x
    h = x
    if pre_layer_norm:
        h = F.layer_norm(h, [_u(x).shape[-1]], ln1_scale, ln1_bias, ln1_epsilon)
    h = F.linear(h, linear1_weight, linear1_bias)
    h = getattr(F, activation)(h)
    h = F.dropout(h, dropout1_rate, training=training, mode=mode)
    h = F.linear(h, linear2_weight, linear2_bias)
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
    """qkv_weight: [3, H, D, E] (reference layout) or [E, 3E] with transpose_qkv_wb=True."""
    t = _u(x)
    B, S, E = t.shape
    h = x
    if pre_layer_norm:
        h = F.layer_norm(h, [E], pre_ln_scale, pre_ln_bias, pre_ln_epsilon)
    w = _u(qkv_weight)
    if transpose_qkv_wb:
        qkv = torch.matmul(_u(h), w)
        if qkv_bias is not None:
            qkv = qkv + _u(qkv_bias)
        H = num_heads
        qkv = qkv.reshape(B, S, 3, H, E // H)
    else:
        _, H, D, _ = w.shape
        qkv = torch.einsum('bse,thde->bsthd', _u(h), w)
        if qkv_bias is not None:
            qkv = qkv + _u(qkv_bias).reshape(1, 1, 3, H, D)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o = F.scaled_dot_product_attention(_w(q), _w(k), _w(v), attn_mask, attn_dropout_rate, False, training)
    o = _w(_u(o).reshape(B, S, -1))
    o = F.linear(o, linear_weight, linear_bias)
    if add_residual:
        o = fused_dropout_add(o, x, dropout_rate, training, mode)
    if not pre_layer_norm:
        o = F.layer_norm(o, [E], ln_scale, ln_bias, ln_epsilon)
    return o


def masked_multihead_attention(x, cache_kv=None, bias=None, src_mask=None, cum_offsets=None, sequence_lengths=None,
                               rotary_tensor=None, beam_cache_offset=None, qkv_out_scale=None, out_shift=None,
                               out_smooth=None, seq_len=1, rotary_emb_dims=0, use_neox_rotary_style=False,
                               compute_dtype='default', out_scale=-1, quant_round_type=1, quant_max_bound=127.0,
                               quant_min_bound=-127.0):
    """Decode-step attention over a [2, B, H, max_len, D] cache (reference masked_multihead_attention)."""
    t = _u(x)
    cache = _u(cache_kv)
    _, B, H, L, D = cache.shape
    qkv = t.reshape(B, 3, H, D)
    if bias is not None:
        qkv = qkv + _u(bias).reshape(1, 3, H, D)
    q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
    lens = _u(sequence_lengths).reshape(-1) if sequence_lengths is not None else torch.zeros(B, dtype=torch.long,
                                                                                             device=t.device)
    ar = torch.arange(B, device=t.device)
    cache[0, ar, :, lens] = k
    cache[1, ar, :, lens] = v
    keys, vals = cache[0], cache[1]
    s = torch.einsum('bhd,bhld->bhl', q.float(), keys.float()) / math.sqrt(D)
    pos = torch.arange(L, device=t.device)[None, None, :]
    s = s.masked_fill(pos > lens[:, None, None], float('-inf'))
    if src_mask is not None:
        s = s + _u(src_mask).reshape(B, 1, -1)[..., :L]
    p = torch.softmax(s, -1)
    o = torch.einsum('bhl,bhld->bhd', p, vals.float()).to(t.dtype)
    return _w(o.reshape(B, H * D)), _w(cache)


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


def fused_ec_moe(x, gate, bmm0_weight, bmm0_bias, bmm1_weight, bmm1_bias, act_type):
    t, g = _u(x), _u(gate)
    probs = torch.softmax(g.float(), -1)
    h = torch.einsum('bsd,edf->bsef', t, _u(bmm0_weight)) + _u(bmm0_bias).reshape(1, 1, *_u(bmm0_bias).shape[-2:])
    h = TF.gelu(h) if act_type == 'gelu' else torch.relu(h)
    o = torch.einsum('bsef,efd->bsed', h, _u(bmm1_weight)) + _u(bmm1_bias).reshape(1, 1, *_u(bmm1_bias).shape[-2:])
    return _w((o * probs.unsqueeze(-1).to(o.dtype)).sum(2))


def blha_get_max_len(seq_lens_encoder, seq_lens_decoder, batch_size):
    return _w(_u(seq_lens_encoder).max().reshape(1)), _w(_u(seq_lens_decoder).max().reshape(1))
