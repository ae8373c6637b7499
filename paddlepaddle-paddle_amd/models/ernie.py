"""ERNIE / BERT encoders (reference models: PaddleNLP ``ErnieModel`` / ``BertModel``).

Post-LN Transformer encoder: word + position + token-type embeddings → LN; each layer
attention → add+LN → GeLU FFN → add+LN (fused add+LayerNorm kernels).  Without a padding mask
the attention runs on csrc/flash_attn.hip; with one it takes the masked SDPA path.
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
class ErnieConfig:
    vocab_size: int = 18000
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    max_position_embeddings: int = 512
    type_vocab_size: int = 4
    initializer_range: float = 0.02
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0


ERNIE_CONFIGS = {
    'ernie-3.0-base': dict(vocab_size=40000, type_vocab_size=4, max_position_embeddings=2048),
    'ernie-1.0-base': dict(),
    'bert-base-uncased': dict(vocab_size=30522, type_vocab_size=2, layer_norm_eps=1e-12),
    'bert-large-uncased': dict(vocab_size=30522, hidden_size=1024, num_hidden_layers=24, num_attention_heads=16,
                               intermediate_size=4096, type_vocab_size=2),
    'ernie-tiny': dict(vocab_size=512, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                       intermediate_size=128, max_position_embeddings=128),
}


def ernie_config(name, **overrides):
    d = dict(ERNIE_CONFIGS[name])
    d.update(overrides)
    return ErnieConfig(**d)


class ErnieEmbeddings(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        init = nn.initializer.TruncatedNormal(0.0, cfg.initializer_range)
        self.word_embeddings = nn.Embedding(cfg.vocab_size, cfg.hidden_size, padding_idx=cfg.pad_token_id,
                                            weight_attr=init)
        self.position_embeddings = nn.Embedding(cfg.max_position_embeddings, cfg.hidden_size, weight_attr=init)
        self.token_type_embeddings = nn.Embedding(cfg.type_vocab_size, cfg.hidden_size, weight_attr=init)
        self.layer_norm = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.dropout = nn.Dropout(cfg.hidden_dropout_prob)

    def forward(self, input_ids, token_type_ids=None, position_ids=None):
        ids = _unwrap(input_ids)
        if position_ids is None:
            position_ids = _wrap(torch.arange(ids.shape[1], device=ids.device).unsqueeze(0).expand_as(ids))
        if token_type_ids is None:
            token_type_ids = _wrap(torch.zeros_like(ids))
        e = self.word_embeddings(input_ids) + self.position_embeddings(position_ids) + \
            self.token_type_embeddings(token_type_ids)
        return self.dropout(self.layer_norm(e))


class ErnieSelfAttention(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.nh = cfg.num_attention_heads
        self.hd = cfg.hidden_size // self.nh
        self.qkv = nn.Linear(cfg.hidden_size, 3 * cfg.hidden_size)
        self.out = nn.Linear(cfg.hidden_size, cfg.hidden_size)
        self.p = cfg.attention_probs_dropout_prob

    def forward(self, x, attn_mask=None):
        t = _unwrap(x)
        B, S, _ = t.shape
        qkv = _unwrap(self.qkv(x)).view(B, S, 3, self.nh, self.hd)
        if attn_mask is None and (not self.training or self.p == 0.0):
            o = F.flash_attn_qkvpacked(_wrap(qkv), causal=False, training=self.training)[0]
            o = _unwrap(o)
        else:
            q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
            m = None
            if attn_mask is not None:
                am = _unwrap(attn_mask)
                m = am.bool() if am.dtype == torch.bool else am.to(q.dtype)
                if m.dim() == 2:  # [B, S] 1 = keep
                    m = m.view(B, 1, 1, S).bool() if m.dtype != torch.bool else m.view(B, 1, 1, S)
            if m is not None and (q.is_cuda or q.is_meta):
                o = F.masked_attention_bhsd(q, k, v, m, self.p if self.training else 0.0).transpose(1, 2)
            else:
                o = TF.scaled_dot_product_attention(q, k, v, attn_mask=m,
                                                    dropout_p=self.p if self.training else 0.0).transpose(1, 2)
        return self.out(_wrap(o.reshape(B, S, -1)))


class ErnieLayer(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.attn = ErnieSelfAttention(cfg)
        self.ln1 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.fc1 = nn.Linear(cfg.hidden_size, cfg.intermediate_size)
        self.fc2 = nn.Linear(cfg.intermediate_size, cfg.hidden_size)
        self.ln2 = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.p = cfg.hidden_dropout_prob
        self.eps = cfg.layer_norm_eps

    def _drop(self, x):
        return F.dropout(x, self.p, training=self.training) if self.p > 0 else x

    def forward(self, x, attn_mask=None):
        a = self._drop(self.attn(x, attn_mask))
        h, _ = IF.fused_layer_norm(a, self.ln1.weight, self.ln1.bias, self.eps, residual=x)
        f = self._drop(self.fc2(F.gelu(self.fc1(h))))
        y, _ = IF.fused_layer_norm(f, self.ln2.weight, self.ln2.bias, self.eps, residual=h)
        return y


class ErnieModel(nn.Layer):
    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.embeddings = ErnieEmbeddings(cfg)
        self.encoder = nn.LayerList([ErnieLayer(cfg) for _ in range(cfg.num_hidden_layers)])
        self.pooler = nn.Linear(cfg.hidden_size, cfg.hidden_size)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        if attention_mask is None:
            ids = _unwrap(input_ids)
            # a static Program cannot branch on data: always build the padding mask there
            if ids.is_meta or (ids == self.config.pad_token_id).any():
                attention_mask = _wrap(ids != self.config.pad_token_id)
        h = self.embeddings(input_ids, token_type_ids, position_ids)
        for layer in self.encoder:
            h = layer(h, attention_mask)
        pooled = F.tanh(self.pooler(_wrap(_unwrap(h)[:, 0])))
        return h, pooled


class ErnieForSequenceClassification(nn.Layer):
    def __init__(self, cfg, num_classes=2, dropout=None):
        super().__init__()
        self.ernie = ErnieModel(cfg)
        self.dropout = nn.Dropout(dropout if dropout is not None else cfg.hidden_dropout_prob)
        self.classifier = nn.Linear(cfg.hidden_size, num_classes)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None):
        _, pooled = self.ernie(input_ids, token_type_ids, position_ids, attention_mask)
        return self.classifier(self.dropout(pooled))


class ErnieForPretraining(nn.Layer):
    """Masked-LM (tied to the word embeddings) + next-sentence heads."""

    def __init__(self, cfg):
        super().__init__()
        self.config = cfg
        self.ernie = ErnieModel(cfg)
        self.transform = nn.Linear(cfg.hidden_size, cfg.hidden_size)
        self.transform_ln = nn.LayerNorm(cfg.hidden_size, epsilon=cfg.layer_norm_eps)
        self.decoder_bias = self.create_parameter([cfg.vocab_size], is_bias=True)
        self.nsp = nn.Linear(cfg.hidden_size, 2)

    def forward(self, input_ids, token_type_ids=None, position_ids=None, attention_mask=None, masked_positions=None):
        h, pooled = self.ernie(input_ids, token_type_ids, position_ids, attention_mask)
        t = _unwrap(h)
        if masked_positions is not None:
            t = t.reshape(-1, t.shape[-1])[_unwrap(masked_positions).reshape(-1)]
        z = self.transform_ln(F.gelu(self.transform(_wrap(t))))
        logits = ops.matmul.matmul(_unwrap(z), _unwrap(self.ernie.embeddings.word_embeddings.weight).t()) + \
            _unwrap(self.decoder_bias)
        return _wrap(logits), self.nsp(pooled)


class ErniePretrainingCriterion(nn.Layer):
    def forward(self, prediction_scores, seq_relationship_score, masked_lm_labels, next_sentence_labels=None):
        lg = _unwrap(prediction_scores).float()
        lm = TF.cross_entropy(lg.reshape(-1, lg.shape[-1]), _unwrap(masked_lm_labels).reshape(-1), ignore_index=-100)
        if next_sentence_labels is None:
            return _wrap(lm)
        ns = TF.cross_entropy(_unwrap(seq_relationship_score).float(), _unwrap(next_sentence_labels).reshape(-1))
        return _wrap(lm + ns)


# BERT shares the architecture
BertConfig, BertModel, BertForSequenceClassification, BertForPretraining = (
    ErnieConfig, ErnieModel, ErnieForSequenceClassification, ErnieForPretraining)
_ = (math, IF, ops)
