"""paddle.incubate.nn fused layers (reference: python/paddle/incubate/nn/layer/{fused_linear,fused_transformer,
fused_dropout_add}.py).  Parameter names/shapes follow the reference."""
import torch

from ...nn.layer.layers import Layer
from ...nn import initializer as I
from ...nn import functional as F
from ...core.tensor import _wrap, _unwrap
from . import functional as IF


class FusedLinear(Layer):
    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, transpose_weight=False, name=None):
        super().__init__()
        shape = [out_features, in_features] if transpose_weight else [in_features, out_features]
        self.weight = self.create_parameter(shape, attr=weight_attr)
        self.bias = self.create_parameter([out_features], attr=bias_attr, is_bias=True)
        self.transpose_weight = transpose_weight

    def forward(self, input):  # noqa: A002
        return IF.fused_linear(input, self.weight, self.bias, self.transpose_weight)


class FusedDropoutAdd(Layer):
    def __init__(self, p=0.5, mode="upscale_in_train", name=None):
        super().__init__()
        self.p, self.mode = p, mode

    def forward(self, x, y):
        return IF.fused_dropout_add(x, y, self.p, self.training, self.mode)


class FusedBiasDropoutResidualLayerNorm(Layer):
    def __init__(self, embed_dim, dropout_rate=0.5, weight_attr=None, bias_attr=None, epsilon=1e-5, name=None):
        super().__init__()
        self.linear_bias = self.create_parameter([embed_dim], attr=bias_attr, is_bias=True)
        self.ln_scale = self.create_parameter([embed_dim], attr=weight_attr, default_initializer=I.Constant(1.0))
        self.ln_bias = self.create_parameter([embed_dim], attr=bias_attr, is_bias=True)
        self.p, self.eps = dropout_rate, epsilon

    def forward(self, x, residual):
        h = IF.fused_dropout_add(_wrap(_unwrap(x) + _unwrap(self.linear_bias)), residual, self.p, self.training)
        return F.layer_norm(h, [_unwrap(h).shape[-1]], self.ln_scale, self.ln_bias, self.eps)


class FusedMultiHeadAttention(Layer):
    def __init__(self, embed_dim, num_heads, dropout_rate=0.5, attn_dropout_rate=0.5, kdim=None, vdim=None,
                 normalize_before=False, need_weights=False, qkv_weight_attr=None, qkv_bias_attr=None,
                 linear_weight_attr=None, linear_bias_attr=None, pre_ln_scale_attr=None, pre_ln_bias_attr=None,
                 ln_scale_attr=None, ln_bias_attr=None, epsilon=1e-5, nranks=1, ring_id=-1, transpose_qkv_wb=False,
                 name=None):
        super().__init__()
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.normalize_before, self.transpose_qkv_wb = normalize_before, transpose_qkv_wb
        if transpose_qkv_wb:
            self.qkv_weight = self.create_parameter([embed_dim, 3 * embed_dim], attr=qkv_weight_attr)
            self.qkv_bias = self.create_parameter([3 * embed_dim], attr=qkv_bias_attr, is_bias=True)
        else:
            self.qkv_weight = self.create_parameter([3, num_heads, self.head_dim, embed_dim], attr=qkv_weight_attr)
            self.qkv_bias = self.create_parameter([3, num_heads, self.head_dim], attr=qkv_bias_attr, is_bias=True)
        self.linear_weight = self.create_parameter([embed_dim, embed_dim], attr=linear_weight_attr)
        self.linear_bias = self.create_parameter([embed_dim], attr=linear_bias_attr, is_bias=True)
        self.pre_ln_scale = self.create_parameter([embed_dim], attr=pre_ln_scale_attr, default_initializer=I.Constant(1.0))
        self.pre_ln_bias = self.create_parameter([embed_dim], attr=pre_ln_bias_attr, is_bias=True)
        self.ln_scale = self.create_parameter([embed_dim], attr=ln_scale_attr, default_initializer=I.Constant(1.0))
        self.ln_bias = self.create_parameter([embed_dim], attr=ln_bias_attr, is_bias=True)
        self.dropout_rate, self.attn_dropout_rate, self.epsilon = dropout_rate, attn_dropout_rate, epsilon

    def forward(self, query, key=None, value=None, attn_mask=None, cache=None):
        return IF.fused_multi_head_attention(
            query, self.qkv_weight, self.linear_weight, self.normalize_before, self.pre_ln_scale, self.pre_ln_bias,
            self.ln_scale, self.ln_bias, self.epsilon, self.qkv_bias, self.linear_bias, cache, attn_mask,
            self.dropout_rate, self.attn_dropout_rate, self.epsilon, self.training, num_heads=self.num_heads,
            transpose_qkv_wb=self.transpose_qkv_wb)


class FusedFeedForward(Layer):
    def __init__(self, d_model, dim_feedforward, dropout_rate=0.1, epsilon=1e-05, activation="relu",
                 act_dropout_rate=None, normalize_before=False, linear1_weight_attr=None, linear1_bias_attr=None,
                 linear2_weight_attr=None, linear2_bias_attr=None, ln1_scale_attr=None, ln1_bias_attr=None,
                 ln2_scale_attr=None, ln2_bias_attr=None, nranks=1, ring_id=-1, name=None):
        super().__init__()
        self._d = d_model
        self.normalize_before, self.activation = normalize_before, activation
        self.dropout_rate = dropout_rate
        self.act_dropout_rate = dropout_rate if act_dropout_rate is None else act_dropout_rate
        self.epsilon = epsilon
        self._linear1_weight = self.create_parameter([d_model, dim_feedforward], attr=linear1_weight_attr)
        self._linear1_bias = self.create_parameter([dim_feedforward], attr=linear1_bias_attr, is_bias=True)
        self._linear2_weight = self.create_parameter([dim_feedforward, d_model], attr=linear2_weight_attr)
        self._linear2_bias = self.create_parameter([d_model], attr=linear2_bias_attr, is_bias=True)
        self._ln1_scale = self.create_parameter([d_model], attr=ln1_scale_attr, default_initializer=I.Constant(1.0))
        self._ln1_bias = self.create_parameter([d_model], attr=ln1_bias_attr, is_bias=True)
        self._ln2_scale = self.create_parameter([d_model], attr=ln2_scale_attr, default_initializer=I.Constant(1.0))
        self._ln2_bias = self.create_parameter([d_model], attr=ln2_bias_attr, is_bias=True)

    def forward(self, src, cache=None):
        return IF.fused_feedforward(src, self._linear1_weight, self._linear2_weight, self._linear1_bias,
                                    self._linear2_bias, self._ln1_scale, self._ln1_bias, self._ln2_scale,
                                    self._ln2_bias, self.act_dropout_rate, self.dropout_rate, self.activation,
                                    self.epsilon, self.epsilon, self.normalize_before, self.training)


class FusedTransformerEncoderLayer(Layer):
    def __init__(self, d_model, nhead, dim_feedforward, dropout_rate=0.1, activation="relu", attn_dropout_rate=None,
                 act_dropout_rate=None, normalize_before=False, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        attn_dropout_rate = dropout_rate if attn_dropout_rate is None else attn_dropout_rate
        self.fused_attn = FusedMultiHeadAttention(d_model, nhead, dropout_rate, attn_dropout_rate,
                                                  normalize_before=normalize_before, transpose_qkv_wb=True)
        self.ffn = FusedFeedForward(d_model, dim_feedforward, dropout_rate, activation=activation,
                                    act_dropout_rate=act_dropout_rate, normalize_before=normalize_before)

    def forward(self, src, src_mask=None, cache=None):
        return self.ffn(self.fused_attn(src, attn_mask=src_mask))


class FusedMultiTransformer(Layer):
    """Stack of pre-LN decoder blocks for inference (reference FusedMultiTransformer): per layer
    ln → fused qkv → (cached) attention → out proj → residual → ln → ffn → residual."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, ln_scale_attrs=None, ln_bias_attrs=None, qkv_weight_attrs=None,
                 qkv_bias_attrs=None, linear_weight_attrs=None, linear_bias_attrs=None, ffn_ln_scale_attrs=None,
                 ffn_ln_bias_attrs=None, ffn1_weight_attrs=None, ffn1_bias_attrs=None, ffn2_weight_attrs=None,
                 ffn2_bias_attrs=None, epsilon=1e-5, num_layers=-1, nranks=1, trans_qkvw=True, ring_id=-1,
                 name=None, **kw):
        super().__init__()
        from ...nn.layer.container import LayerList
        self.num_layers = num_layers if num_layers > 0 else 1
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.activation, self.epsilon = activation, epsilon
        self.ln_scales, self.ln_biases, self.qkv_weights, self.qkv_biases = [], [], [], []
        self.linear_weights, self.linear_biases, self.ffn_ln_scales, self.ffn_ln_biases = [], [], [], []
        self.ffn1_weights, self.ffn1_biases, self.ffn2_weights, self.ffn2_biases = [], [], [], []
        for i in range(self.num_layers):
            mk = self.create_parameter
            self.ln_scales.append(mk([embed_dim], default_initializer=I.Constant(1.0)))
            self.ln_biases.append(mk([embed_dim], is_bias=True))
            self.qkv_weights.append(mk([3, num_heads, self.head_dim, embed_dim]))
            self.qkv_biases.append(mk([3, num_heads, self.head_dim], is_bias=True))
            self.linear_weights.append(mk([embed_dim, embed_dim]))
            self.linear_biases.append(mk([embed_dim], is_bias=True))
            self.ffn_ln_scales.append(mk([embed_dim], default_initializer=I.Constant(1.0)))
            self.ffn_ln_biases.append(mk([embed_dim], is_bias=True))
            self.ffn1_weights.append(mk([embed_dim, dim_feedforward]))
            self.ffn1_biases.append(mk([dim_feedforward], is_bias=True))
            self.ffn2_weights.append(mk([dim_feedforward, embed_dim]))
            self.ffn2_biases.append(mk([embed_dim], is_bias=True))
            for n, lst in (('ln_scale', self.ln_scales), ('ln_bias', self.ln_biases), ('qkv_weight', self.qkv_weights),
                           ('qkv_bias', self.qkv_biases), ('linear_weight', self.linear_weights),
                           ('linear_bias', self.linear_biases), ('ffn_ln_scale', self.ffn_ln_scales),
                           ('ffn_ln_bias', self.ffn_ln_biases), ('ffn1_weight', self.ffn1_weights),
                           ('ffn1_bias', self.ffn1_biases), ('ffn2_weight', self.ffn2_weights),
                           ('ffn2_bias', self.ffn2_biases)):
                self.add_parameter(f"{n}_{i}", lst[-1])

    def forward(self, src, attn_mask=None, caches=None, time_step=None, **kw):
        x = src
        B, S, E = _unwrap(x).shape
        new_caches = []
        for i in range(self.num_layers):
            h = F.layer_norm(x, [E], self.ln_scales[i], self.ln_biases[i], self.epsilon)
            w = _unwrap(self.qkv_weights[i])
            qkv = torch.einsum('bse,thde->bsthd', _unwrap(h), w) + _unwrap(self.qkv_biases[i]).reshape(1, 1, 3,
                                                                                                    self.num_heads,
                                                                                                    self.head_dim)
            q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
            if caches is not None:
                ck = _unwrap(caches[i])  # [2, B, S_past, H, D]
                k = torch.cat([ck[0], k], 1)
                v = torch.cat([ck[1], v], 1)
                new_caches.append(_wrap(torch.stack([k, v])))
            causal = attn_mask is None
            o = F.scaled_dot_product_attention(_wrap(q), _wrap(k), _wrap(v), attn_mask, 0.0, causal, False)
            o = F.linear(_wrap(_unwrap(o).reshape(B, S, E)), self.linear_weights[i], self.linear_biases[i])
            x = _wrap(_unwrap(x) + _unwrap(o))
            h = F.layer_norm(x, [E], self.ffn_ln_scales[i], self.ffn_ln_biases[i], self.epsilon)
            h = F.linear(h, self.ffn1_weights[i], self.ffn1_biases[i])
            h = getattr(F, self.activation)(h)
            h = F.linear(h, self.ffn2_weights[i], self.ffn2_biases[i])
            x = _wrap(_unwrap(x) + _unwrap(h))
        return (x, new_caches) if caches is not None else x
