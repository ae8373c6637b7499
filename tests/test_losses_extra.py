"""rnnt_loss against the reference op test's fixtures, adaptive log-softmax vs a numpy reference,
FusedEcMoe layer.  Reference: nn/functional/loss.py:1983 / :4289, incubate/nn/layer/fused_ec_moe.py."""
import os
import sys

import numpy as np
import pytest
import scipy.special as sps

import paddle
import paddle.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import fixtures_rnnt as FX  # noqa: E402


@pytest.mark.parametrize("dtype", ['float32', 'float64'])
def test_rnnt_loss_matches_reference_fixture(dtype):
    acts = paddle.to_tensor(FX.ACTS.astype(dtype), stop_gradient=False)
    lab = paddle.to_tensor(FX.LABELS)
    tl, ul = paddle.to_tensor(FX.LOGIT_LENS), paddle.to_tensor(FX.LABEL_LENS)
    loss = F.rnnt_loss(acts, lab, tl, ul, blank=0, fastemit_lambda=0.0, reduction='none')
    np.testing.assert_allclose(loss.numpy(), FX.LOSS, rtol=1e-5)
    loss.sum().backward()
    np.testing.assert_allclose(acts.grad.numpy(), FX.GRAD, atol=1e-5)


def test_rnnt_reductions_layer_and_fastemit():
    acts = paddle.to_tensor(FX.ACTS.astype('float64'), stop_gradient=False)
    args = (paddle.to_tensor(FX.LABELS), paddle.to_tensor(FX.LOGIT_LENS), paddle.to_tensor(FX.LABEL_LENS))
    m = F.rnnt_loss(acts, *args, fastemit_lambda=0.0)
    s = F.rnnt_loss(acts, *args, fastemit_lambda=0.0, reduction='sum')
    np.testing.assert_allclose(float(m), FX.LOSS.sum() / 3, rtol=1e-6)
    np.testing.assert_allclose(float(s), FX.LOSS.sum(), rtol=1e-6)
    layer = paddle.nn.RNNTLoss(blank=0, fastemit_lambda=0.01, reduction='sum')
    fe = layer(acts, *args)
    np.testing.assert_allclose(float(fe), FX.LOSS.sum(), rtol=1e-6)  # FastEmit leaves the value
    fe.backward()
    g_fe = acts.grad.numpy().copy()
    acts.clear_gradient()
    F.rnnt_loss(acts, *args, fastemit_lambda=0.0, reduction='sum').backward()
    assert not np.allclose(g_fe, acts.grad.numpy())  # ... and rescales the emission gradients


def test_rnnt_shorter_sequences_ignore_padding():
    acts = FX.ACTS.astype('float64')
    full = F.rnnt_loss(paddle.to_tensor(acts[:1, :3]), paddle.to_tensor(FX.LABELS[:1]),
                       paddle.to_tensor([3]), paddle.to_tensor([2]), fastemit_lambda=0.0, reduction='none')
    padded = np.concatenate([acts[:1, :3], np.full((1, 1, 3, 3), 5.0)], 1)
    got = F.rnnt_loss(paddle.to_tensor(padded), paddle.to_tensor(FX.LABELS[:1]), paddle.to_tensor([3]),
                      paddle.to_tensor([2]), fastemit_lambda=0.0, reduction='none')
    np.testing.assert_allclose(got.numpy(), full.numpy())


def _np_adaptive(x, y, hw, hb, tails, cutoffs):
    head = x @ hw + (hb if hb is not None else 0)
    hl = sps.log_softmax(head, -1)
    out = np.zeros(len(y))
    for r in range(len(y)):
        if y[r] < cutoffs[0]:
            out[r] = hl[r, y[r]]
            continue
        for i in range(1, len(cutoffs)):
            if cutoffs[i - 1] <= y[r] < cutoffs[i]:
                w0, w1 = tails[i - 1]
                cl = sps.log_softmax((x[r] @ w0) @ w1)
                out[r] = hl[r, cutoffs[0] + i - 1] + cl[y[r] - cutoffs[i - 1]]
    return out


def test_adaptive_log_softmax_with_loss():
    paddle.seed(0)
    m = paddle.nn.AdaptiveLogSoftmaxWithLoss(16, 20, [4, 10], div_value=2.0, head_bias=True)
    x = np.random.RandomState(0).randn(9, 16).astype('float32')
    y = np.array([0, 3, 4, 9, 10, 19, 2, 15, 7])
    out, loss = m(paddle.to_tensor(x), paddle.to_tensor(y))
    tails = [(w0.numpy(), w1.numpy()) for w0, w1 in m.tail_weights]
    ref = _np_adaptive(x, y, m.head_weight.numpy(), m.head_bias.numpy(), tails, [4, 10, 20])
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(float(loss), -ref.mean(), rtol=1e-5)
    lp = m.log_prob(paddle.to_tensor(x)).numpy()
    np.testing.assert_allclose(np.exp(lp).sum(-1), 1.0, rtol=1e-5)
    np.testing.assert_allclose(lp[np.arange(9), y], ref, rtol=1e-5, atol=1e-6)
    assert len(m.parameters()) == 6  # head w/b + 2 x (proj, out), real paddle Parameters
    loss.backward()
    assert m.head_weight.grad is not None


def test_fused_ec_moe_layer():
    paddle.seed(0)
    moe = paddle.incubate.nn.FusedEcMoe(16, 32, 4, act_type='gelu')
    x = paddle.randn([2, 5, 16])
    gate = paddle.randn([2, 5, 4])
    y = moe(x, gate)
    assert y.shape == [2, 5, 16]
    with pytest.raises(NotImplementedError):
        paddle.incubate.nn.FusedEcMoe(16, 32, 4, act_type='silu')
