"""Model zoo: Llama (GQA + RoPE) and ERNIE/BERT train on CPU; the fused paths are GPU-tested."""
import numpy as np
import pytest
import torch

import paddle
from paddle.models import llama_config, LlamaForCausalLM, ernie_config, ErnieForSequenceClassification, \
    ErnieForPretraining, ErniePretrainingCriterion


def test_llama_tiny_trains_and_rope_matches_reference():
    paddle.seed(0)
    cfg = llama_config('llama-tiny')
    m = LlamaForCausalLM(cfg)
    opt = paddle.optimizer.AdamW(3e-3, parameters=m.parameters())
    ids = paddle.to_tensor(np.random.RandomState(0).randint(0, cfg.vocab_size, (4, 33)))
    x, y = ids[:, :-1], ids[:, 1:]
    losses = []
    for _ in range(12):
        loss = m.loss(m(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] - 0.5, losses
    out = m.generate(x[:1, :5], max_new_tokens=3)
    assert out.shape == [1, 8]
    # rope: rotate-half form equals complex multiplication
    from paddle.models.llama import _rope_ref
    from paddle.ops.rope import rope_tables
    cos, sin = rope_tables(16, 8)
    q = torch.randn(1, 16, 2, 8)
    r = _rope_ref(q, cos, sin)
    qc = torch.complex(q[..., :4], q[..., 4:])
    rc = qc * torch.complex(cos, sin).view(1, 16, 1, 4)
    torch.testing.assert_close(r, torch.cat([rc.real, rc.imag], -1))


def test_ernie_cls_and_pretraining():
    paddle.seed(0)
    cfg = ernie_config('ernie-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = ErnieForSequenceClassification(cfg, num_classes=3)
    ids = paddle.to_tensor(np.random.RandomState(1).randint(1, cfg.vocab_size, (4, 16)))
    ids._t[0, 12:] = 0  # padding → masked attention path
    logits = m(ids)
    assert logits.shape == [4, 3]
    pm = ErnieForPretraining(cfg)
    pred, nsp = pm(ids, masked_positions=paddle.to_tensor([1, 5, 17]))
    assert pred.shape == [3, cfg.vocab_size] and nsp.shape == [4, 2]
    loss = ErniePretrainingCriterion()(pred, nsp, paddle.to_tensor([3, 4, 5]), paddle.to_tensor([0, 1, 0, 1]))
    loss.backward()
    assert pm.ernie.embeddings.word_embeddings.weight.grad is not None


@pytest.mark.gpu
def test_llama_tiny_gpu_matches_cpu_reference():
    paddle.seed(0)
    cfg = llama_config('llama-tiny')
    m = LlamaForCausalLM(cfg)
    ids = paddle.randint(0, cfg.vocab_size, [2, 64])
    out_gpu = m(ids)
    paddle.ops.set_enabled(False)
    try:
        out_ref = m(ids)
    finally:
        paddle.ops.set_enabled(True)
    assert float((out_gpu - out_ref).abs().max()) < 2e-3 * float(out_ref.abs().max()) + 1e-3
