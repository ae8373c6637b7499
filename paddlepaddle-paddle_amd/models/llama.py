"""Llama-2 family causal LM (reference model: PaddleNLP ``LlamaForCausalLM``, trained with the
reference's fleet hybrid parallel / sharding stack).

MI355X mapping per decoder block:
  add + RMSNorm           → csrc/norm.hip (residual fused; returns the new residual stream)
  q/k/v projection        → one hipBLASLt GEMM into a packed [B, S, Hq + 2·Hkv, D] buffer
  RoPE                    → csrc/embed_rope_optim.hip (fp32 cos/sin tables built once)
  attention (GQA)         → csrc/flash_attn.hip on strided views, dK/dV summed per kv group
  gate/up projection      → one GEMM into [.., 2·I]; SwiGLU → csrc/act.hip
"""
import math
from dataclasses import dataclass

import torch
import torch.nn.functional as TF

from .. import nn
from ..nn import functional as F
from ..core.tensor import _wrap, _unwrap
from ..incubate.nn import functional as IF
from .. import ops


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    initializer_range: float = 0.02
    tie_word_embeddings: bool = False
    use_recompute: bool = False


LLAMA_CONFIGS = {
    'llama2-7b': dict(),
    'llama2-13b': dict(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40, num_attention_heads=40,
                       num_key_value_heads=40),
    'llama2-70b': dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
                       num_key_value_heads=8),
    'llama3-8b': dict(vocab_size=128256, intermediate_size=14336, num_key_value_heads=8, rope_theta=500000.0,
                      max_position_embeddings=8192),
    'llama-tiny': dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=256),
}


def llama_config(name, **overrides):
    d = dict(LLAMA_CONFIGS[name])
    d.update(overrides)
    return LlamaConfig(**d)


def _rope_ref(x, cos, sin):
    """Reference rotate-half RoPE (CPU / fallback path): x [B, S, H, D], cos/sin [S, D/2]."""
    S = x.shape[1]
    c = cos[:S].to(x.dtype).view(1, S, 1, -1)
    s = sin[:S].to(x.dtype).view(1, S, 1, -1)
    x1, x2 = x.chunk(2, -1)
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1)


class LlamaAttention(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.cfg = cfg
        self.nh, self.nkv = cfg.num_attention_heads, cfg.num_key_value_heads
        self.hd = cfg.hidden_size // self.nh
        init = nn.initializer.Normal(0.0, cfg.initializer_range)
        self.qkv_proj = nn.Linear(cfg.hidden_size, (self.nh + 2 * self.nkv) * self.hd, weight_attr=init,
                                  bias_attr=False)
        self.o_proj = nn.Linear(self.nh * self.hd, cfg.hidden_size, weight_attr=nn.initializer.Normal(
            0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers)), bias_attr=False)

    def forward(self, x, position_ids=None):
        t = _unwrap(x)
        B, S, _ = t.shape
        qkv = _unwrap(self.qkv_proj(x)).view(B, S, self.nh + 2 * self.nkv, self.hd)
        q, k, v = qkv[:, :, :self.nh], qkv[:, :, self.nh:self.nh + self.nkv], qkv[:, :, self.nh + self.nkv:]
        cos, sin = ops.rope.rope_tables(self.cfg.max_position_embeddings, self.hd, self.cfg.rope_theta, t.device)
        pos = _unwrap(position_ids) if position_ids is not None else None
        if ops.use_hip(t) and ops.flash_attn.qkv_rope_flash_ok(qkv, self.nh, self.nkv):
            # RoPE read from / dQKV written into the fused projection's layout (ops/flash_attn.py
            # _QKVRopeFlash): no slice copies, no zero-filled per-slice gradients to add up
            o = ops.flash_attn.qkv_rope_flash(qkv, self.nh, self.nkv, cos, sin, pos, causal=True)
            return self.o_proj(_wrap(o.reshape(B, S, -1)))
        if ops.use_hip(t):
            q = ops.rope.apply_rope(q, cos, sin, pos)
            k = ops.rope.apply_rope(k, cos, sin, pos)
        else:
            if pos is not None:
                cos, sin = cos[pos], sin[pos]
                q = torch.cat([_rope_ref(q[b:b + 1], cos[b], sin[b]) for b in range(B)])
                k = torch.cat([_rope_ref(k[b:b + 1], cos[b], sin[b]) for b in range(B)])
            else:
                q, k = _rope_ref(q, cos, sin), _rope_ref(k, cos, sin)
        o = F.flash_attention(_wrap(q), _wrap(k), _wrap(v), causal=True, training=self.training)[0]
        return self.o_proj(_wrap(_unwrap(o).reshape(B, S, -1)))


class LlamaMLP(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        init = nn.initializer.Normal(0.0, cfg.initializer_range)
        self.gate_up_proj = nn.Linear(cfg.hidden_size, 2 * cfg.intermediate_size, weight_attr=init, bias_attr=False)
        self.down_proj = nn.Linear(cfg.intermediate_size, cfg.hidden_size, weight_attr=nn.initializer.Normal(
            0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers)), bias_attr=False)

    def forward(self, x):
        return self.down_proj(F.swiglu(self.gate_up_proj(x)))


class LlamaDecoderLayer(nn.Layer):
    """Pre-RMSNorm block; ``forward(x, residual)`` fuses every residual add into the next
    RMSNorm kernel and returns (mlp_out, residual_stream)."""

    def __init__(self, cfg):
        super().__init__()
        self.input_layernorm = nn.RMSNorm(cfg.hidden_size, epsilon=cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg)
        self.post_attention_layernorm = nn.RMSNorm(cfg.hidden_size, epsilon=cfg.rms_norm_eps)
        self.mlp = LlamaMLP(cfg)
        self.eps = cfg.rms_norm_eps

    def forward(self, x, residual=None, position_ids=None):
        if residual is None:
            a, h = self.input_layernorm(x), x
        else:
            a, h = IF.fused_rms_norm(x, self.input_layernorm.weight, None, self.eps, residual=residual)
        attn = self.self_attn(a, position_ids)
        b, h = IF.fused_rms_norm(attn, self.post_attention_layernorm.weight, None, self.eps, residual=h)
        return self.mlp(b), h


class LlamaModel(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size,
                                         weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))
        self.layers = nn.LayerList([LlamaDecoderLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.norm = nn.RMSNorm(cfg.hidden_size, epsilon=cfg.rms_norm_eps)

    def forward(self, input_ids, position_ids=None):
        x = self.embed_tokens(input_ids)
        out, res = x, None
        for layer in self.layers:
            if self.config.use_recompute and self.training:
                from ..distributed.fleet.recompute import recompute
                out, res = recompute(layer, out, res, position_ids)
            else:
                out, res = layer(out, res, position_ids)
        y, _ = IF.fused_rms_norm(out, self.norm.weight, None, self.config.rms_norm_eps, residual=res)
        return y


class LlamaForCausalLM(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.llama = LlamaModel(cfg)
        if not cfg.tie_word_embeddings:
            self.lm_head = nn.Linear(cfg.hidden_size, cfg.vocab_size, bias_attr=False,
                                     weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))

    def forward(self, input_ids, position_ids=None):
        h = self.llama(input_ids, position_ids)
        if self.config.tie_word_embeddings:
            return _wrap(ops.matmul.matmul(_unwrap(h), _unwrap(self.llama.embed_tokens.weight).t()))
        return self.lm_head(h)

    def loss(self, logits, labels, ignore_index=-100):
        lg, lab = _unwrap(logits), _unwrap(labels)
        if ops.use_hip(lg):
            per_tok = ops.xent.softmax_cross_entropy(lg.reshape(-1, lg.shape[-1]), lab.reshape(-1), ignore_index,
                                                     inplace_grad=True)
            valid = (lab.reshape(-1) != ignore_index).sum().clamp(min=1)
            return _wrap(per_tok.sum() / valid)
        return _wrap(TF.cross_entropy(lg.reshape(-1, lg.shape[-1]).float(), lab.reshape(-1),
                                      ignore_index=ignore_index))

    @torch.no_grad()
    def generate(self, input_ids, max_new_tokens=16, temperature=0.0):
        """Greedy / temperature sampling without a KV cache (reference-style generate for tests)."""
        ids = _unwrap(input_ids)
        for _ in range(max_new_tokens):
            logits = _unwrap(self(_wrap(ids)))[:, -1].float()
            if temperature > 0:
                nxt = torch.multinomial(torch.softmax(logits / temperature, -1), 1)
            else:
                nxt = logits.argmax(-1, keepdim=True)
            ids = torch.cat([ids, nxt.to(ids.dtype)], 1)
        return _wrap(ids)
