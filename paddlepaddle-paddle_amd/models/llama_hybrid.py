"""Llama-2 for Fleet hybrid parallelism: tensor parallel (Megatron column/row split of attention
heads and MLP), pipeline parallel (PipelineLayer of LayerDescs), and — through the fleet
sharding stage — optimizer-state sharding (BASELINE config "Llama-2 13B HybridParallel
TP=2 x PP=2 x sharding-2").

Reference: PaddleNLP ``LlamaForCausalLMPipe`` / ``LlamaAttention(config.tensor_parallel_degree)``
built on python/paddle/distributed/fleet/layers/mpu/mp_layers.py (ColumnParallelLinear:334,
RowParallelLinear:541, VocabParallelEmbedding:47, ParallelCrossEntropy:742) and
meta_parallel/parallel_layers/pp_layers.py (LayerDesc, PipelineLayer).

Per rank: q/k/v/gate/up are ColumnParallelLinear (no gather: each rank owns nh/mp heads and
inter/mp MLP columns), o/down are RowParallelLinear (input already parallel; one all-reduce each),
the embedding is vocab-parallel and the LM head a column-parallel GEMM feeding the vocab-parallel
cross entropy — two all-reduces per decoder layer forward, the Megatron minimum.
``load_full_weights`` shards a single-device ``LlamaForCausalLM`` into this layout (used by the
equivalence tests, and to start hybrid training from a dense checkpoint).
"""
import math

import torch

from .. import nn
from ..nn import functional as F
from ..core.tensor import _wrap, _unwrap
from .. import ops
from .llama import LlamaConfig, llama_config, _rope_ref  # noqa: F401


def _mpu():
    from ..distributed.fleet.layers.mpu import mp_layers
    return mp_layers


class LlamaAttentionTP(nn.Layer):
    def __init__(self, cfg, mp_group=None):
        super().__init__()
        mpu = _mpu()
        self.cfg = cfg
        self.hd = cfg.hidden_size // cfg.num_attention_heads
        init = nn.initializer.Normal(0.0, cfg.initializer_range)
        h = cfg.hidden_size
        self.q_proj = mpu.ColumnParallelLinear(h, cfg.num_attention_heads * self.hd, weight_attr=init, has_bias=False,
                                               gather_output=False, mp_group=mp_group)
        self.k_proj = mpu.ColumnParallelLinear(h, cfg.num_key_value_heads * self.hd, weight_attr=init,
                                               has_bias=False, gather_output=False, mp_group=mp_group)
        self.v_proj = mpu.ColumnParallelLinear(h, cfg.num_key_value_heads * self.hd, weight_attr=init,
                                               has_bias=False, gather_output=False, mp_group=mp_group)
        self.o_proj = mpu.RowParallelLinear(cfg.num_attention_heads * self.hd, h, has_bias=False,
                                            input_is_parallel=True, mp_group=mp_group, weight_attr=nn.initializer.Normal(
                                                0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers)))
        mp = self.q_proj.world_size
        self.nh, self.nkv = cfg.num_attention_heads // mp, cfg.num_key_value_heads // mp

    def forward(self, x):
        t = _unwrap(x)
        B, S, _ = t.shape
        q = _unwrap(self.q_proj(x)).view(B, S, self.nh, self.hd)
        k = _unwrap(self.k_proj(x)).view(B, S, self.nkv, self.hd)
        v = _unwrap(self.v_proj(x)).view(B, S, self.nkv, self.hd)
        cos, sin = ops.rope.rope_tables(self.cfg.max_position_embeddings, self.hd, self.cfg.rope_theta, t.device)
        if ops.use_hip(t):
            q, k = ops.rope.apply_rope(q, cos, sin, None), ops.rope.apply_rope(k, cos, sin, None)
        else:
            q, k = _rope_ref(q, cos, sin), _rope_ref(k, cos, sin)
        o = F.flash_attention(_wrap(q), _wrap(k), _wrap(v), causal=True, training=self.training)[0]
        return self.o_proj(_wrap(_unwrap(o).reshape(B, S, -1)))


class LlamaMLPTP(nn.Layer):
    def __init__(self, cfg, mp_group=None):
        super().__init__()
        mpu = _mpu()
        init = nn.initializer.Normal(0.0, cfg.initializer_range)
        h, f = cfg.hidden_size, cfg.intermediate_size
        self.gate_proj = mpu.ColumnParallelLinear(h, f, weight_attr=init, has_bias=False, gather_output=False,
                                                  mp_group=mp_group)
        self.up_proj = mpu.ColumnParallelLinear(h, f, weight_attr=init, has_bias=False, gather_output=False,
                                                mp_group=mp_group)
        self.down_proj = mpu.RowParallelLinear(f, h, has_bias=False, input_is_parallel=True, mp_group=mp_group,
                                               weight_attr=nn.initializer.Normal(
                                                   0.0, cfg.initializer_range / math.sqrt(2.0 * cfg.num_hidden_layers)))

    def forward(self, x):
        return self.down_proj(F.swiglu(self.gate_proj(x), self.up_proj(x)))


class LlamaDecoderLayerTP(nn.Layer):
    """Pre-RMSNorm block with the residual adds explicit (a pipeline stage passes one tensor)."""

    def __init__(self, cfg, mp_group=None):
        super().__init__()
        self.input_layernorm = nn.RMSNorm(cfg.hidden_size, epsilon=cfg.rms_norm_eps)
        self.self_attn = LlamaAttentionTP(cfg, mp_group)
        self.post_attention_layernorm = nn.RMSNorm(cfg.hidden_size, epsilon=cfg.rms_norm_eps)
        self.mlp = LlamaMLPTP(cfg, mp_group)

    def forward(self, x):
        h = x + self.self_attn(self.input_layernorm(x))
        return h + self.mlp(self.post_attention_layernorm(h))


class LlamaEmbeddingPipe(nn.Layer):
    def __init__(self, cfg, mp_group=None):
        super().__init__()
        self.embed_tokens = _mpu().VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, mp_group=mp_group,
                                                          weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))

    def forward(self, ids):
        return self.embed_tokens(ids)


class LlamaLMHeadPipe(nn.Layer):
    def __init__(self, cfg, mp_group=None):
        super().__init__()
        self.norm = nn.RMSNorm(cfg.hidden_size, epsilon=cfg.rms_norm_eps)
        self.lm_head = _mpu().ColumnParallelLinear(cfg.hidden_size, cfg.vocab_size, has_bias=False,
                                                   gather_output=False, mp_group=mp_group,
                                                   weight_attr=nn.initializer.Normal(0.0, cfg.initializer_range))

    def forward(self, x):
        return self.lm_head(self.norm(x))


class LlamaPretrainingCriterionTP(nn.Layer):
    """Mean token loss over vocab-parallel logits (ParallelCrossEntropy)."""

    def __init__(self, mp_group=None, ignore_index=-100):
        super().__init__()
        self.xent = _mpu().ParallelCrossEntropy(mp_group=mp_group, ignore_index=ignore_index)
        self.ignore_index = ignore_index

    def forward(self, logits, labels):
        per_tok = _unwrap(self.xent(logits, labels))
        lab = _unwrap(labels)
        valid = (lab != self.ignore_index).sum().clamp(min=1)
        return _wrap(per_tok.sum() / valid)


def LlamaForCausalLMPipe(cfg, num_stages=None, topology=None, num_virtual_pipeline_stages=None, seg_method="uniform"):
    """PipelineLayer of [embedding, decoder x L, norm + head] with the vocab-parallel loss."""
    from ..distributed.fleet import meta_parallel as mpp
    descs = [mpp.LayerDesc(LlamaEmbeddingPipe, cfg)]
    descs += [mpp.LayerDesc(LlamaDecoderLayerTP, cfg) for _ in range(cfg.num_hidden_layers)]
    descs.append(mpp.LayerDesc(LlamaLMHeadPipe, cfg))
    return mpp.PipelineLayer(descs, num_stages=num_stages, topology=topology, seg_method=seg_method,
                             loss_fn=LlamaPretrainingCriterionTP(),
                             num_virtual_pipeline_stages=num_virtual_pipeline_stages)


# ------------------------------------------------------------------ dense -> hybrid weights
def _col(t, r, n):
    return t.chunk(n, dim=1)[r]


def _row(t, r, n):
    return t.chunk(n, dim=0)[r]


def load_full_weights(pipe, full, mp_rank, mp_size):
    """Copy a single-device ``LlamaForCausalLM`` (fused qkv / gate_up layout) into this rank's
    pipeline stage(s) and tensor-parallel shards."""
    cfg = full.config
    hd = cfg.hidden_size // cfg.num_attention_heads
    nq, nk = cfg.num_attention_heads * hd, cfg.num_key_value_heads * hd
    f = cfg.intermediate_size
    owned = [i for lo, hi in pipe._chunk_ranges for i in range(lo, hi)]
    L = cfg.num_hidden_layers
    with torch.no_grad():
        for layer, gi in zip(pipe.run_function, owned):
            if gi == 0:
                w = _unwrap(full.llama.embed_tokens.weight)
                per = layer.embed_tokens.weight._t.shape[0]
                _unwrap(layer.embed_tokens.weight).copy_(w[mp_rank * per:(mp_rank + 1) * per])
            elif gi == L + 1:
                _unwrap(layer.norm.weight).copy_(_unwrap(full.llama.norm.weight))
                head = _unwrap(full.lm_head.weight) if not cfg.tie_word_embeddings else \
                    _unwrap(full.llama.embed_tokens.weight).t()
                _unwrap(layer.lm_head.weight).copy_(_col(head, mp_rank, mp_size))
            else:
                src = full.llama.layers[gi - 1]
                qkv = _unwrap(src.self_attn.qkv_proj.weight)
                q, k, v = qkv[:, :nq], qkv[:, nq:nq + nk], qkv[:, nq + nk:]
                a = layer.self_attn
                _unwrap(a.q_proj.weight).copy_(_col(q, mp_rank, mp_size))
                _unwrap(a.k_proj.weight).copy_(_col(k, mp_rank, mp_size))
                _unwrap(a.v_proj.weight).copy_(_col(v, mp_rank, mp_size))
                _unwrap(a.o_proj.weight).copy_(_row(_unwrap(src.self_attn.o_proj.weight), mp_rank, mp_size))
                gu = _unwrap(src.mlp.gate_up_proj.weight)
                _unwrap(layer.mlp.gate_proj.weight).copy_(_col(gu[:, :f], mp_rank, mp_size))
                _unwrap(layer.mlp.up_proj.weight).copy_(_col(gu[:, f:], mp_rank, mp_size))
                _unwrap(layer.mlp.down_proj.weight).copy_(_row(_unwrap(src.mlp.down_proj.weight), mp_rank, mp_size))
                _unwrap(layer.input_layernorm.weight).copy_(_unwrap(src.input_layernorm.weight))
                _unwrap(layer.post_attention_layernorm.weight).copy_(_unwrap(src.post_attention_layernorm.weight))
