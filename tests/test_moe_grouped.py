"""MoE expert compute as batched GEMMs (no per-expert Python loop): the grouped path of MoELayer
equals the per-expert loop (forward, input and parameter gradients), structure detection rejects
non-FFN experts, and fused_ec_moe equals its dense formula.  CPU (the GPU run takes the same code
onto the hand-written batched GEMM, tests/test_hip_matmul.py)."""
import pytest
import torch

import paddle
from paddle.incubate.distributed.models.moe import MoELayer, NaiveGate
from paddle.incubate.distributed.models import moe as M


class FFN(paddle.nn.Layer):
    def __init__(self, d, f, act):
        super().__init__()
        self.htoh4 = paddle.nn.Linear(d, f)
        self.h4toh = paddle.nn.Linear(f, d)
        self.act = act

    def forward(self, x):
        return self.h4toh(self.act(self.htoh4(x)))


class Odd(paddle.nn.Layer):
    def __init__(self, d):
        super().__init__()
        self.a = paddle.nn.Linear(d, d)
        self.b = paddle.nn.Linear(d, d)

    def forward(self, x):
        return self.b(x) + self.a(x)  # not an FFN chain


@pytest.mark.parametrize('act,name', [(paddle.nn.functional.relu, 'relu'), (paddle.nn.functional.gelu, 'gelu'),
                                      (paddle.nn.functional.silu, 'silu')])
def test_grouped_experts_match_loop(act, name):
    d, f, E = 16, 32, 4
    res = []
    for grouped in (True, False):
        paddle.seed(1)
        experts = [FFN(d, f, act) for _ in range(E)]
        layer = MoELayer(d, experts, gate=NaiveGate(d, E, 1, topk=2))
        if not grouped:
            layer._grouped = {True: False, False: False}
        x = paddle.to_tensor(torch.randn(3, 7, d, generator=torch.Generator().manual_seed(2)))
        x.stop_gradient = False
        y = layer(x)
        (y ** 2).sum().backward()
        if grouped:
            assert layer._grouped[True] == (0, name)
        res.append((y.numpy(), x.grad.numpy(), [e.htoh4.weight.grad.numpy() for e in experts]))
    (ya, ga, wa), (yb, gb, wb) = res
    assert abs(ya - yb).max() < 1e-5
    assert abs(ga - gb).max() < 1e-5
    for a, b in zip(wa, wb):
        assert abs(a - b).max() < 1e-5


def test_detection_rejects_non_ffn():
    paddle.seed(0)
    layer = MoELayer(8, [Odd(8) for _ in range(2)], gate=NaiveGate(8, 2, 1, topk=1))
    layer(paddle.randn([2, 3, 8]))
    assert layer._grouped[True] is False


class FFNDrop(paddle.nn.Layer):
    def __init__(self, d, f):
        super().__init__()
        self.fc1 = paddle.nn.Linear(d, f)
        self.drop = paddle.nn.Dropout(0.5)
        self.fc2 = paddle.nn.Linear(f, d)

    def forward(self, x):
        return self.fc2(self.drop(paddle.nn.functional.relu(self.fc1(x))))


def test_detection_rejects_dropout_expert_probed_in_eval():
    """An expert with a Dropout between its Linears matches the FFN formula in eval mode; the
    grouped path must not be taken (it would skip the dropout once the layer trains)."""
    paddle.seed(0)
    experts = [FFNDrop(8, 16) for _ in range(2)]
    layer = MoELayer(8, experts, gate=NaiveGate(8, 2, 1, topk=1))
    layer.eval()
    layer(paddle.randn([2, 3, 8]))
    assert layer._grouped[False] is False
    layer.train()
    x = paddle.randn([4, 8, 8])
    y1, y2 = layer(x).numpy(), layer(x).numpy()
    assert abs(y1 - y2).max() > 0  # dropout is live in training forwards


def test_fused_ec_moe_dense_formula():
    paddle.seed(0)
    B, S, D, F, E = 2, 5, 16, 32, 3
    x, gate = torch.randn(B, S, D), torch.randn(B, S, E)
    w0, b0 = torch.randn(E, D, F), torch.randn(E, F)
    w1, b1 = torch.randn(E, F, D), torch.randn(E, D)
    y = paddle.incubate.nn.functional.fused_ec_moe(*[paddle.to_tensor(t) for t in (x, gate, w0, b0, w1, b1)],
                                                   'gelu')
    p = torch.softmax(gate, -1)
    ref = sum(p[..., e:e + 1] * (torch.nn.functional.gelu(x @ w0[e] + b0[e]) @ w1[e] + b1[e]) for e in range(E))
    assert torch.allclose(y._t, ref, atol=1e-4)
