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
        return IF.fused_bias_dropout_residual_layer_norm(x, residual, self.linear_bias, self.ln_scale, self.ln_bias,
                                                         self.p, self.eps, self.training)


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
    """Stack of transformer blocks for generation (reference incubate/nn/layer/fused_transformer.py:994):
    parameters per layer in the reference shapes (qkv [3, H, D, E] with trans_qkvw, or
    [(H + 2 Hkv), D, E] with gqa_group_size), forward = incubate.nn.functional.fused_multi_transformer
    with caches [2, B, Hkv, max_len, D] updated in place and ``time_step`` selecting the decode step."""

    def __init__(self, embed_dim, num_heads, dim_feedforward, dropout_rate=0.0, activation="gelu",
                 normalize_before=True, ln_scale_attrs=None, ln_bias_attrs=None, qkv_weight_attrs=None,
                 qkv_bias_attrs=None, linear_weight_attrs=None, linear_bias_attrs=None, ffn_ln_scale_attrs=None,
                 ffn_ln_bias_attrs=None, ffn1_weight_attrs=None, ffn1_bias_attrs=None, ffn2_weight_attrs=None,
                 ffn2_bias_attrs=None, epsilon=1e-5, residual_alpha=1.0, num_layers=-1, nranks=1, trans_qkvw=True,
                 ring_id=-1, norm_type="layernorm", use_neox_rotary_style=False, gqa_group_size=-1, name=None):
        super().__init__()
        assert embed_dim > 0 and num_heads > 0 and dim_feedforward > 0
        if num_layers < 0:
            num_layers = len(qkv_weight_attrs) if isinstance(qkv_weight_attrs, (list, tuple)) else 1
        self.num_layers = num_layers
        self.embed_dim, self.num_heads = embed_dim, num_heads
        self.head_dim = embed_dim // num_heads
        self.activation, self.epsilon, self.residual_alpha = activation, epsilon, residual_alpha
        self.normalize_before, self.trans_qkvw, self.norm_type = normalize_before, trans_qkvw, norm_type
        self.use_neox_rotary_style, self.gqa_group_size = use_neox_rotary_style, gqa_group_size
        self.dropout_rate = dropout_rate
        H, D, E = num_heads, self.head_dim, embed_dim
        nqkv = (H + 2 * gqa_group_size) if gqa_group_size > 0 else None
        ffn1_out = dim_feedforward * 2 if activation in ('swiglu', 'geglu') else dim_feedforward
        names = ['ln_scale', 'ln_bias', 'qkv_weight', 'qkv_bias', 'linear_weight', 'linear_bias', 'ffn_ln_scale',
                 'ffn_ln_bias', 'ffn1_weight', 'ffn1_bias', 'ffn2_weight', 'ffn2_bias']
        plural = {n: (n[:-4] + 'biases' if n.endswith('bias') else n + 's') for n in names}
        for n in names:
            setattr(self, plural[n], [])

        def attr(a, i):
            return a[i] if isinstance(a, (list, tuple)) else a

        for i in range(num_layers):
            mk = self.create_parameter
            if nqkv is not None:
                qkv_shape = [nqkv, D, E] if trans_qkvw else [E, nqkv, D]
                qkvb_shape = [nqkv * D]
            else:
                qkv_shape = [3, H, D, E] if trans_qkvw else [E, 3, H, D]
                qkvb_shape = [3, H, D]
            vals = [mk([E], attr=attr(ln_scale_attrs, i), default_initializer=I.Constant(1.0)),
                    mk([E], attr=attr(ln_bias_attrs, i), is_bias=True),
                    mk(qkv_shape, attr=attr(qkv_weight_attrs, i)),
                    mk(qkvb_shape, attr=attr(qkv_bias_attrs, i), is_bias=True),
                    mk([H * D, E], attr=attr(linear_weight_attrs, i)),
                    mk([E], attr=attr(linear_bias_attrs, i), is_bias=True),
                    mk([E], attr=attr(ffn_ln_scale_attrs, i), default_initializer=I.Constant(1.0)),
                    mk([E], attr=attr(ffn_ln_bias_attrs, i), is_bias=True),
                    mk([E, ffn1_out], attr=attr(ffn1_weight_attrs, i)),
                    mk([ffn1_out], attr=attr(ffn1_bias_attrs, i), is_bias=True),
                    mk([dim_feedforward, E], attr=attr(ffn2_weight_attrs, i)),
                    mk([E], attr=attr(ffn2_bias_attrs, i), is_bias=True)]
            for n, v in zip(names, vals):
                getattr(self, plural[n]).append(v)
                self.add_parameter(f"{n}_{i}", v)

    def forward(self, src, attn_mask=None, caches=None, pre_caches=None, rotary_embs=None, rotary_emb_dims=0,
                beam_offset=None, seq_lens=None, time_step=None):
        if caches is not None:
            assert len(caches) == len(self.qkv_weights)
        return IF.fused_multi_transformer(
            src, self.ln_scales, self.ln_biases, self.qkv_weights, self.qkv_biases, self.linear_weights,
            self.linear_biases, self.ffn_ln_scales, self.ffn_ln_biases, self.ffn1_weights, self.ffn1_biases,
            self.ffn2_weights, self.ffn2_biases, pre_layer_norm=self.normalize_before, epsilon=self.epsilon,
            residual_alpha=self.residual_alpha, cache_kvs=caches, beam_offset=beam_offset, pre_caches=pre_caches,
            seq_lens=seq_lens, rotary_embs=rotary_embs, time_step=time_step, attn_mask=attn_mask,
            dropout_rate=self.dropout_rate, rotary_emb_dims=rotary_emb_dims, activation=self.activation,
            training=self.training, trans_qkvw=self.trans_qkvw, norm_type=self.norm_type,
            use_neox_rotary_style=self.use_neox_rotary_style, gqa_group_size=self.gqa_group_size)



class FusedEcMoe(Layer):
    """Reference incubate/nn/layer/fused_ec_moe.py: experts [E, d_model, d_ff] / [E, d_ff, d_model]
    with [E, 1, d] biases; forward(x [B, S, d_model], gate [B, S, E]) -> [B, S, d_model]."""

    def __init__(self, hidden_size, inter_size, num_experts, act_type, weight_attr=None, bias_attr=None):
        super().__init__()
        if act_type not in ('gelu', 'relu'):
            raise NotImplementedError("Currently only support `gelu`, `relu`. ")
        self.bmm_weight0 = self.create_parameter([num_experts, hidden_size, inter_size], attr=weight_attr)
        self.bmm_bias0 = self.create_parameter([num_experts, 1, inter_size], attr=bias_attr, is_bias=True)
        self.bmm_weight1 = self.create_parameter([num_experts, inter_size, hidden_size], attr=weight_attr)
        self.bmm_bias1 = self.create_parameter([num_experts, 1, hidden_size], attr=bias_attr, is_bias=True)
        self.act_type = act_type

    def forward(self, x, gate):
        return IF.fused_ec_moe(x, gate, self.bmm_weight0, self.bmm_bias0, self.bmm_weight1, self.bmm_bias1,
                               self.act_type)
