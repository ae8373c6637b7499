"""Transformer layers (reference: python/paddle/nn/layer/transformer.py).

Attention runs through ``F.scaled_dot_product_attention`` (BSHD layout) so unmasked
attention on HIP tensors takes the MFMA flash-attention kernel.
"""
import copy
import collections

import torch

from .layers import Layer
from .common import Linear, Dropout
from .norm import LayerNorm
from .container import LayerList
from .. import functional as F
from ...core.tensor import Tensor, _wrap, _unwrap


def _convert_attention_mask(attn_mask, dtype):
    if attn_mask is None:
        return None
    m = _unwrap(attn_mask)
    if m.dtype == torch.bool:
        return m  # True = attend (paddle convention == torch SDPA bool convention)
    return m.to(dtype)


class MultiHeadAttention(Layer):
    Cache = collections.namedtuple("Cache", ["k", "v"])
    StaticCache = collections.namedtuple("StaticCache", ["k", "v"])

    def __init__(self, embed_dim, num_heads, dropout=0.0, kdim=None, vdim=None, need_weights=False, weight_attr=None,
                 bias_attr=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.kdim, self.vdim = kdim or embed_dim, vdim or embed_dim
        self.dropout, self.need_weights = dropout, need_weights
        self.head_dim = embed_dim // num_heads
        assert self.head_dim * num_heads == embed_dim, "embed_dim must be divisible by num_heads"
        self.q_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)
        self.k_proj = Linear(self.kdim, embed_dim, weight_attr, bias_attr)
        self.v_proj = Linear(self.vdim, embed_dim, weight_attr, bias_attr)
        self.out_proj = Linear(embed_dim, embed_dim, weight_attr, bias_attr)

    def _split(self, x):
        t = _unwrap(x)
        return t.reshape(t.shape[0], t.shape[1], self.num_heads, self.head_dim)

    def _prepare_qkv(self, query, key, value, cache=None):
        q = self._split(self.q_proj(query))
        if isinstance(cache, self.StaticCache):
            k, v = _unwrap(cache.k), _unwrap(cache.v)
        else:
            k = self._split(self.k_proj(key))
            v = self._split(self.v_proj(value))
        if isinstance(cache, self.Cache):
            k = torch.cat([_unwrap(cache.k), k], 1)
            v = torch.cat([_unwrap(cache.v), v], 1)
            cache = self.Cache(_wrap(k), _wrap(v))
        return q, k, v, cache

    def gen_cache(self, key, value=None, type=Cache):  # noqa: A002
        if type == MultiHeadAttention.StaticCache:
            k = _wrap(self._split(self.k_proj(key)))
            v = _wrap(self._split(self.v_proj(value if value is not None else key)))
            return self.StaticCache(k, v)
        if value is None:
            b = _unwrap(key).shape[0]
            z = torch.zeros(b, 0, self.num_heads, self.head_dim, dtype=_unwrap(key).dtype, device=_unwrap(key).device)
            return self.Cache(_wrap(z), _wrap(z.clone()))
        return self.Cache(key, value)

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        key = query if key is None else key
        value = query if value is None else value
        q, k, v, cache = self._prepare_qkv(query, key, value, cache)
        mask = _convert_attention_mask(attn_mask, q.dtype)
        weights = None
        if self.need_weights:
            qh, kh, vh = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
            s = qh @ kh.transpose(-1, -2) / (self.head_dim ** 0.5)
            if mask is not None:
                s = s.masked_fill(~mask, float('-inf')) if mask.dtype == torch.bool else s + mask
            p = torch.softmax(s, -1)
            weights = _wrap(p)
            p = torch.nn.functional.dropout(p, self.dropout, self.training)
            o = (p @ vh).transpose(1, 2)
        else:
            o = _unwrap(F.scaled_dot_product_attention(_wrap(q), _wrap(k), _wrap(v), _wrap(mask) if mask is not None else None,
                                                       self.dropout, False, self.training))
        out = self.out_proj(_wrap(o.reshape(o.shape[0], o.shape[1], self.embed_dim)))
        outs = [out]
        if self.need_weights:
            outs.append(weights)
        if cache is not None:
            outs.append(cache)
        return out if len(outs) == 1 else tuple(outs)


def _act_fn(name):
    return getattr(F, name)


class TransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, dropout=attn_dropout, weight_attr=weight_attr,
                                            bias_attr=bias_attr)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(act_dropout, mode="upscale_in_train")
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout, mode="upscale_in_train")
        self.dropout2 = Dropout(dropout, mode="upscale_in_train")
        self.activation = _act_fn(activation)

    def forward(self, src, src_mask=None, cache=None):
        residual = src
        if self.normalize_before:
            src = self.norm1(src)
        if cache is None:
            src = self.self_attn(src, src, src, src_mask)
        else:
            src, incremental_cache = self.self_attn(src, src, src, src_mask, cache)
        src = residual + self.dropout1(src)
        if not self.normalize_before:
            src = self.norm1(src)
        residual = src
        if self.normalize_before:
            src = self.norm2(src)
        src = self.linear2(self.dropout(self.activation(self.linear1(src))))
        src = residual + self.dropout2(src)
        if not self.normalize_before:
            src = self.norm2(src)
        return src if cache is None else (src, incremental_cache)

    def gen_cache(self, src):
        return self.self_attn.gen_cache(src, type=self.self_attn.Cache)


class TransformerEncoder(Layer):
    def __init__(self, encoder_layer, num_layers, norm=None, enable_recompute=False):
        super().__init__()
        self.layers = LayerList([(encoder_layer if i == 0 else copy.deepcopy(encoder_layer)) for i in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm
        self.enable_recompute = enable_recompute

    def forward(self, src, src_mask=None, cache=None):
        output = src
        new_caches = []
        for i, mod in enumerate(self.layers):
            if cache is None:
                if self.enable_recompute and self.training:
                    from ...distributed.fleet.recompute import recompute
                    output = recompute(mod, output, src_mask)
                else:
                    output = mod(output, src_mask=src_mask)
            else:
                output, new_cache = mod(output, src_mask=src_mask, cache=cache[i])
                new_caches.append(new_cache)
        if self.norm is not None:
            output = self.norm(output)
        return output if cache is None else (output, new_caches)

    def gen_cache(self, src):
        return [layer.gen_cache(src) for layer in self.layers]


class TransformerDecoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout=0.1, activation="relu", attn_dropout=None,
                 act_dropout=None, normalize_before=False, weight_attr=None, bias_attr=None, layer_norm_eps=1e-5):
        super().__init__()
        attn_dropout = dropout if attn_dropout is None else attn_dropout
        act_dropout = dropout if act_dropout is None else act_dropout
        self.normalize_before = normalize_before
        self.self_attn = MultiHeadAttention(d_model, nhead, dropout=attn_dropout, weight_attr=weight_attr,
                                            bias_attr=bias_attr)
        self.cross_attn = MultiHeadAttention(d_model, nhead, dropout=attn_dropout, weight_attr=weight_attr,
                                             bias_attr=bias_attr)
        self.linear1 = Linear(d_model, dim_feedforward, weight_attr, bias_attr)
        self.dropout = Dropout(act_dropout, mode="upscale_in_train")
        self.linear2 = Linear(dim_feedforward, d_model, weight_attr, bias_attr)
        self.norm1 = LayerNorm(d_model, layer_norm_eps)
        self.norm2 = LayerNorm(d_model, layer_norm_eps)
        self.norm3 = LayerNorm(d_model, layer_norm_eps)
        self.dropout1 = Dropout(dropout, mode="upscale_in_train")
        self.dropout2 = Dropout(dropout, mode="upscale_in_train")
        self.dropout3 = Dropout(dropout, mode="upscale_in_train")
        self.activation = _act_fn(activation)

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        residual = tgt
        if self.normalize_before:
            tgt = self.norm1(tgt)
        if cache is None:
            tgt = self.self_attn(tgt, tgt, tgt, tgt_mask, None)
        else:
            tgt, incremental_cache = self.self_attn(tgt, tgt, tgt, tgt_mask, cache[0])
        tgt = residual + self.dropout1(tgt)
        if not self.normalize_before:
            tgt = self.norm1(tgt)
        residual = tgt
        if self.normalize_before:
            tgt = self.norm2(tgt)
        if cache is None:
            tgt = self.cross_attn(tgt, memory, memory, memory_mask, None)
        else:
            tgt, static_cache = self.cross_attn(tgt, memory, memory, memory_mask, cache[1])
        tgt = residual + self.dropout2(tgt)
        if not self.normalize_before:
            tgt = self.norm2(tgt)
        residual = tgt
        if self.normalize_before:
            tgt = self.norm3(tgt)
        tgt = self.linear2(self.dropout(self.activation(self.linear1(tgt))))
        tgt = residual + self.dropout3(tgt)
        if not self.normalize_before:
            tgt = self.norm3(tgt)
        return tgt if cache is None else (tgt, (incremental_cache, static_cache))

    def gen_cache(self, memory):
        incremental_cache = self.self_attn.gen_cache(memory, type=self.self_attn.Cache)
        static_cache = self.cross_attn.gen_cache(memory, memory, type=self.cross_attn.StaticCache)
        return incremental_cache, static_cache


class TransformerDecoder(Layer):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = LayerList([(decoder_layer if i == 0 else copy.deepcopy(decoder_layer)) for i in range(num_layers)])
        self.num_layers = num_layers
        self.norm = norm

    def forward(self, tgt, memory, tgt_mask=None, memory_mask=None, cache=None):
        output = tgt
        new_caches = []
        for i, mod in enumerate(self.layers):
            if cache is None:
                output = mod(output, memory, tgt_mask=tgt_mask, memory_mask=memory_mask, cache=None)
            else:
                output, new_cache = mod(output, memory, tgt_mask=tgt_mask, memory_mask=memory_mask, cache=cache[i])
                new_caches.append(new_cache)
        if self.norm is not None:
            output = self.norm(output)
        return output if cache is None else (output, new_caches)

    def gen_cache(self, memory, do_zip=False):
        cache = [layer.gen_cache(memory) for layer in self.layers]
        if do_zip:
            cache = list(zip(*cache))
        return cache


class Transformer(Layer):
    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6, dim_feedforward=2048,
                 dropout=0.1, activation="relu", attn_dropout=None, act_dropout=None, normalize_before=False,
                 weight_attr=None, bias_attr=None, custom_encoder=None, custom_decoder=None):
        super().__init__()
        if custom_encoder is not None:
            self.encoder = custom_encoder
        else:
            enc = TransformerEncoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout,
                                          act_dropout, normalize_before, weight_attr, bias_attr)
            self.encoder = TransformerEncoder(enc, num_encoder_layers, LayerNorm(d_model) if normalize_before else None)
        if custom_decoder is not None:
            self.decoder = custom_decoder
        else:
            dec = TransformerDecoderLayer(d_model, nhead, dim_feedforward, dropout, activation, attn_dropout,
                                          act_dropout, normalize_before, weight_attr, bias_attr)
            self.decoder = TransformerDecoder(dec, num_decoder_layers, LayerNorm(d_model) if normalize_before else None)
        self.d_model, self.nhead = d_model, nhead

    def forward(self, src, tgt, src_mask=None, tgt_mask=None, memory_mask=None):
        memory = self.encoder(src, src_mask=src_mask)
        return self.decoder(tgt, memory, tgt_mask=tgt_mask, memory_mask=memory_mask)

    @staticmethod
    def generate_square_subsequent_mask(length):
        m = torch.triu(torch.full((length, length), float('-inf')), 1)
        from ...core.place import current_device
        return _wrap(m.to(current_device()))
