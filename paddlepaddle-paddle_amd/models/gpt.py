"""GPT (GPT-2/GPT-3 family) for causal-LM pretraining.

Reference model: PaddleNLP/PaddleFleetX ``GPTForPretraining`` (the model behind the
reference's GPT-3 1.3B sharding benchmark): learned absolute positions, pre-LayerNorm
decoder blocks, fused QKV projection, GeLU MLP (4h), tied input/output embeddings.

MI355X mapping (per decoder block):
  add+LayerNorm         → one HIP kernel (csrc/norm.hip, residual fused, fp32 stats)
  QKV / out / fc1 / fc2 → hand-written 8-phase MFMA GEMMs (csrc/gemm8.hip), bias fused in the epilogue
  attention             → csrc/flash_attn.hip on strided q/k/v views of the QKV output
                          (no transposes, no S×S matrix)
  GeLU (+ fc1 bias)     → csrc/act.hip; backward writes dx and reduces the bias grad in one pass
  dropout + residual + LayerNorm (+ out-proj bias) → ONE csrc/norm.hip kernel each way
                          (mask regenerated in backward from a counter hash)
  LM head + loss        → hand-written GEMMs (tied, E.grad accumulated in place) + csrc/softmax_xent.hip
"""
from ..framework.flags import pa_flag  # noqa: E402
import math
import os
from dataclasses import dataclass

import torch

from .. import nn
from ..nn import functional as F
from ..core.tensor import Tensor, _wrap, _unwrap
from ..incubate.nn import functional as IF
from .. import ops


@dataclass
class GPTConfig:
    vocab_size: int = 50304
    hidden_size: int = 2048
    num_hidden_layers: int = 24
    num_attention_heads: int = 16
    intermediate_size: int = 8192
    max_position_embeddings: int = 1024
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.0
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-5
    use_recompute: bool = False
    fused_ce_inplace: bool = True


GPT_CONFIGS = {
    'gpt3-125m': dict(hidden_size=768, num_hidden_layers=12, num_attention_heads=12, intermediate_size=3072),
    'gpt3-350m': dict(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096),
    'gpt3-1.3b': dict(hidden_size=2048, num_hidden_layers=24, num_attention_heads=16, intermediate_size=8192),
    'gpt3-2.7b': dict(hidden_size=2560, num_hidden_layers=32, num_attention_heads=32, intermediate_size=10240),
    'gpt3-6.7b': dict(hidden_size=4096, num_hidden_layers=32, num_attention_heads=32, intermediate_size=16384),
    'gpt3-13b': dict(hidden_size=5120, num_hidden_layers=40, num_attention_heads=40, intermediate_size=20480),
    'gpt-tiny': dict(vocab_size=512, hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                     intermediate_size=512, max_position_embeddings=128),
}


def gpt_config(name, **overrides):
    d = dict(GPT_CONFIGS[name])
    d.update(overrides)
    return GPTConfig(**d)


# fc2 bias handed to the next fused dropout + residual + LayerNorm (its gradient reduced in that
# kernel's backward pass) instead of a GEMM bias epilogue + a column-sum pass (tests switch it)
DEFER_FC2_BIAS = pa_flag('defer_fc2_bias')


def _normal(std):
    return nn.initializer.Normal(0.0, std)


class GPTAttention(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        h = cfg.hidden_size
        self.num_heads = cfg.num_attention_heads
        self.head_dim = h // self.num_heads
        self.qkv_proj = nn.Linear(h, 3 * h, weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))
        self.out_proj = nn.Linear(h, h, weight_attr=nn.initializer.Normal(
            0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers)))
        self.attn_dropout = cfg.attention_probs_dropout_prob

    def core(self, x):
        """Attention up to (not including) the output projection: [B, S, hidden]."""
        t = _unwrap(x)
        B, S, _ = t.shape
        qkv = _unwrap(self.qkv_proj(x)).view(B, S, 3, self.num_heads, self.head_dim)
        # packed: q/k/v are strided BSHD views for the kernel and dQ/dK/dV land in one buffer
        o = F.flash_attn_qkvpacked(_wrap(qkv), dropout=self.attn_dropout, causal=True, training=self.training)[0]
        return _wrap(_unwrap(o).reshape(B, S, -1))

    def forward(self, x):
        return self.out_proj(self.core(x))


class GPTMLP(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.fc1 = nn.Linear(cfg.hidden_size, cfg.intermediate_size,
                             weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))
        self.fc2 = nn.Linear(cfg.intermediate_size, cfg.hidden_size, weight_attr=nn.initializer.Normal(
            0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers)))

    def forward(self, x):
        return self.fc2(F.gelu(self.fc1(x), approximate=True))


class DeferredBias:
    """A bias Parameter still to be added to a block's output (deliberately not a Tensor, so layer
    hooks that act on tensor outputs — e.g. the sharding engine's — leave it alone)."""
    __slots__ = ('param',)

    def __init__(self, param):
        self.param = param


class GPTDecoderLayer(nn.Layer):
    """Pre-LN block.  ``forward(x, residual)`` takes the *un-added* sublayer output of the
    previous block and the residual stream, so every residual add is fused into the next
    LayerNorm kernel: returns (mlp_out, residual_stream)."""

    def __init__(self, cfg):
        super().__init__()
        h = cfg.hidden_size
        self.ln1 = nn.LayerNorm(h, epsilon=cfg.layer_norm_eps)
        self.attn = GPTAttention(cfg)
        self.ln2 = nn.LayerNorm(h, epsilon=cfg.layer_norm_eps)
        self.mlp = GPTMLP(cfg)
        self.p = cfg.hidden_dropout_prob

    def _drop(self, x):
        return F.dropout(x, self.p, training=self.training) if self.p > 0 else x

    def _fused(self, x):
        return self.training and ops.fused.dropout_add_norm_ok(_unwrap(x), None, self.p) and \
            ops.fused.bias_act_ok(_unwrap(x), self.mlp.fc1.bias)

    def forward(self, x, residual=None, x_bias=None, defer_bias=False):
        """Returns (out, residual_stream); with ``defer_bias=True`` (the GPT model's own loop)
        (out, residual_stream, DeferredBias or None): the fc2 bias may be left to the consumer,
        which hands it to the next fused dropout + residual + LayerNorm kernel (bias added there,
        its gradient reduced in that kernel's backward: no separate column-sum over the MLP
        output).  ``x_bias``: the previous block's DeferredBias for ``x``.  Not deferred when the
        bias can be released after this block's forward (sharding stage-3 units)."""
        xb = x_bias.param if x_bias is not None else None
        if self._fused(x):
            out, h, ob = self._forward_fused(x, residual, xb)
        else:
            if xb is not None:
                x = _wrap(_unwrap(x) + xb._t)
            out, h = self._forward_plain(x, residual)
            ob = None
        if defer_bias:
            return out, h, (DeferredBias(ob) if ob is not None else None)
        if ob is not None:
            out = _wrap(_unwrap(out) + ob._t)
        return out, h

    def _forward_plain(self, x, residual):
        if residual is None:
            a, h = self.ln1(x), x
        else:
            a, h = IF.fused_layer_norm(self._drop(x), self.ln1.weight, self.ln1.bias, self.ln1._epsilon,
                                       residual=residual)
        attn = self.attn(a)
        b, h = IF.fused_layer_norm(self._drop(attn), self.ln2.weight, self.ln2.bias, self.ln2._epsilon, residual=h)
        return self.mlp(b), h

    def _forward_fused(self, x, residual, x_bias=None):
        """Training path on the HIP kernels: dropout + residual add + LayerNorm is one kernel each
        way, the out-projection, fc1 and fc2 biases are applied (and their gradients reduced) inside
        the consuming kernels, so those GEMMs run without a bias epilogue.  Returns
        (out, residual, out_bias) — the fc2 bias is deferred to the next norm (forward_deferred)."""
        fz = ops.fused
        if residual is None:
            if x_bias is not None:
                x = _wrap(_unwrap(x) + x_bias._t)
            a, h = self.ln1(x), x
        else:
            a, h = fz.dropout_add_norm(_unwrap(x), x_bias, _unwrap(residual), self.ln1.weight._t, self.ln1.bias._t,
                                       self.ln1._epsilon, self.p)
            a, h = _wrap(a), _wrap(h)
        o = F.linear(self.attn.core(a), self.attn.out_proj.weight, None)
        b, h = fz.dropout_add_norm(_unwrap(o), self.attn.out_proj.bias, _unwrap(h), self.ln2.weight._t,
                                   self.ln2.bias._t, self.ln2._epsilon, self.p)
        m = self.mlp
        ob = m.fc2.bias if (DEFER_FC2_BIAS and m.fc2.bias is not None
                            and not m.fc2.bias.__dict__.get('_releasable', False)) else None
        if ops.linear.mlp_gelu_ok(b, m.fc1.weight, m.fc1.bias, m.fc2.weight):  # GELU in the GEMM epilogues
            y = ops.linear.mlp_gelu(b, m.fc1.weight, m.fc1.bias, m.fc2.weight, None if ob is not None else m.fc2.bias)
            return _wrap(y), _wrap(h), ob
        z = F.linear(_wrap(b), m.fc1.weight, None)
        g = fz.bias_act(_unwrap(z), m.fc1.bias, 'gelu_tanh')
        if ob is not None:
            return F.linear(_wrap(g), m.fc2.weight, None), _wrap(h), ob
        return m.fc2(_wrap(g)), _wrap(h), None


class GPTEmbeddings(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.word_embeddings = nn.Embedding(cfg.vocab_size, cfg.hidden_size,
                                            weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))
        self.position_embeddings = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size,
                                                weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))
        self.p = cfg.hidden_dropout_prob

    def forward(self, input_ids, position_ids=None):
        ids = _unwrap(input_ids)
        if position_ids is None:
            position_ids = _wrap(torch.arange(ids.shape[1], device=ids.device).unsqueeze(0).expand_as(ids))
        e = self.word_embeddings(input_ids) + self.position_embeddings(position_ids)
        return F.dropout(e, self.p, training=self.training) if self.p > 0 else e


class GPTModel(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.embeddings = GPTEmbeddings(cfg)
        self.layers = nn.LayerList([GPTDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.final_norm = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.p = cfg.hidden_dropout_prob

    def forward(self, input_ids, position_ids=None):
        x = self.embeddings(input_ids, position_ids)
        out, res, ob = x, None, None  # ob: the previous block's deferred fc2 bias (forward_deferred)
        for layer in self.layers:
            if self.config.use_recompute and self.training:
                from ..distributed.fleet.recompute import recompute
                if ob is not None:
                    out, ob = _wrap(_unwrap(out) + ob.param._t), None
                out, res = recompute(layer, out, res)
            else:
                out, res, ob = layer(out, res, ob, defer_bias=True)
        if res is not None and self.training and ops.fused.dropout_add_norm_ok(_unwrap(out), None, self.p):
            y, _ = ops.fused.dropout_add_norm(_unwrap(out), ob.param if ob is not None else None, _unwrap(res),
                                              self.final_norm.weight._t, self.final_norm.bias._t,
                                              self.final_norm._epsilon, self.p)
            return _wrap(y)
        if ob is not None:
            out = _wrap(_unwrap(out) + ob.param._t)
        if self.p > 0:
            out = F.dropout(out, self.p, training=self.training)
        y, _ = IF.fused_layer_norm(out, self.final_norm.weight, self.final_norm.bias, self.final_norm._epsilon,
                                   residual=res)
        return y


class GPTForPretraining(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.gpt = GPTModel(cfg)

    def forward(self, input_ids, position_ids=None):
        h = self.gpt(input_ids, position_ids)
        w = self.gpt.embeddings.word_embeddings.weight
        t = _unwrap(h)
        if t.is_cuda and ops.use_hip(t) and t.dtype == torch.bfloat16 and _unwrap(w).dtype == torch.bfloat16:
            from ..ops.linear import tied_head  # hand-written GEMMs, in-place E.grad accumulate
            return _wrap(tied_head(t, w))
        return _wrap(ops.matmul.matmul(t, _unwrap(w).t()))  # tied LM head

    def loss(self, logits, labels):
        lg = _unwrap(logits)
        lab = _unwrap(labels)
        if ops.use_hip(lg):
            per_tok = ops.xent.softmax_cross_entropy(lg.reshape(-1, lg.shape[-1]), lab.reshape(-1),
                                                     inplace_grad=self.config.fused_ce_inplace)
            return _wrap(per_tok.mean())
        return F.cross_entropy(logits, labels)


class GPTPretrainingCriterion(nn.Layer):
    def __init__(self, cfg=None, ignore_index=-100):
        super().__init__()
        self.ignore_index = ignore_index

    def forward(self, logits, labels, loss_mask=None):
        lg = _unwrap(logits)
        lab = _unwrap(labels)
        if ops.use_hip(lg):
            per_tok = ops.xent.softmax_cross_entropy(lg.reshape(-1, lg.shape[-1]), lab.reshape(-1),
                                                     self.ignore_index)
        else:
            per_tok = torch.nn.functional.cross_entropy(lg.reshape(-1, lg.shape[-1]).float(), lab.reshape(-1),
                                                        ignore_index=self.ignore_index, reduction='none')
        if loss_mask is not None:
            m = _unwrap(loss_mask).reshape(-1).float()
            return _wrap((per_tok * m).sum() / m.sum().clamp_min(1))
        return _wrap(per_tok.mean())
