"""incubate fused_gate_attention / fused_dot_product_attention against the reference's pseudo
code (fused_gate_attention.py:19 docstring) and a plain SDPA, on CPU (the GPU run of the same ops
lands on the hand-written GEMM / flash kernels)."""
import math

import numpy as np
import pytest
import torch

import paddle
import paddle.incubate.nn.functional as IF


def _gate_ref(q_data, m_data, qw, kw, vw, gw, gb, ow, ob, nb, mask, gating):
    c = qw.shape[-1]
    q = torch.einsum('nbqa,ahc->nbqhc', q_data, qw) * c ** -0.5
    k = torch.einsum('nbka,ahc->nbkhc', m_data, kw)
    v = torch.einsum('nbka,ahc->nbkhc', m_data, vw)
    logits = torch.einsum('nbqhc,nbkhc->nbhqk', q, k) + mask
    if nb is not None:
        logits = logits + nb
    w = torch.softmax(logits, -1)
    avg = torch.einsum('nbhqk,nbkhc->nbqhc', w, v)
    if gating:
        gv = torch.sigmoid(torch.einsum('nbqc,chv->nbqhv', q_data, gw) + gb)
        avg = avg * gv
    return torch.einsum('nbqhc,hco->nbqo', avg, ow) + ob


@pytest.mark.parametrize('merge', [True, False])
@pytest.mark.parametrize('gating', [True, False])
def test_fused_gate_attention(merge, gating):
    g = torch.Generator().manual_seed(0)
    B, msa, res, qd, H, c = 2, 3, 5, 8, 4, 6
    x = torch.randn(B, msa, res, qd, generator=g)
    qkv = torch.randn(3, H, c, qd, generator=g) * 0.3
    gw, gb = torch.randn(qd, H, c, generator=g) * 0.3, torch.randn(H, c, generator=g)
    ow, ob = torch.randn(H, c, qd, generator=g) * 0.3, torch.randn(qd, generator=g)
    nb = torch.randn(B, 1, H, res, res, generator=g)
    mask = torch.randn(B, msa, 1, 1, res, generator=g)
    qw, kw, vw = (qkv[i].permute(2, 0, 1).contiguous() for i in range(3))  # [qd, H, c]
    T = paddle.to_tensor
    if merge:
        out = IF.fused_gate_attention(T(x), qkv_weight=T(qkv), gate_linear_weight=T(gw), gate_linear_bias=T(gb),
                                      out_linear_weight=T(ow), out_linear_bias=T(ob), nonbatched_bias=T(nb),
                                      attn_mask=T(mask), has_gating=gating, merge_qkv=True)
    else:
        out = IF.fused_gate_attention(T(x), T(x), query_weight=T(qw), key_weight=T(kw), value_weight=T(vw),
                                      gate_linear_weight=T(gw), gate_linear_bias=T(gb), out_linear_weight=T(ow),
                                      out_linear_bias=T(ob), nonbatched_bias=T(nb), attn_mask=T(mask),
                                      has_gating=gating, merge_qkv=False)
    ref = _gate_ref(x, x, qw, kw, vw, gw, gb, ow, ob, nb, mask, gating)
    assert out.shape == list(ref.shape)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('causal', [False, True])
def test_fused_dot_product_attention(causal):
    g = torch.Generator().manual_seed(1)
    B, S, H, D = 2, 16, 2, 8
    q, k, v = (torch.randn(B, S, H, D, generator=g) for _ in range(3))
    keep = torch.rand(B, 1, S, S, generator=g) > 0.3
    keep[..., 0] = True
    out, sm = IF.fused_dot_product_attention(paddle.to_tensor(q), paddle.to_tensor(k), paddle.to_tensor(v),
                                             paddle.to_tensor(keep.int()), 1 / math.sqrt(D), 0.0, False, causal,
                                             return_softmax=True)
    s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(D)
    m = torch.ones(S, S, dtype=torch.bool).tril() if causal else keep
    s = s.masked_fill(~m, float('-inf'))
    p = torch.softmax(s, -1)
    ref = torch.einsum('bhqk,bkhd->bqhd', p, v)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(sm.numpy(), p.numpy(), rtol=1e-4, atol=1e-6)
