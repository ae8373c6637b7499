"""CPU checks of the matmul routing logic of ops/matmul.py (the GPU numerics are in
tests/test_hip_matmul.py): einsum lowering to one batched GEMM, broadcast batch strides, gradient
reduction over broadcast dims — with the kernel call replaced by torch.matmul."""
import pytest
import torch

from paddle.ops import matmul as hm


@pytest.fixture
def routed(monkeypatch):
    calls = []

    def raw(a, b):
        calls.append((tuple(a.shape), tuple(b.shape)))
        return torch.matmul(a, b)
    monkeypatch.setattr(hm, '_use', lambda *ts: True)
    monkeypatch.setattr(hm, '_matmul_raw', raw)
    return calls


@pytest.mark.parametrize('eq,sx,sy', [
    ('bij,jk->bik', (3, 4, 5), (5, 6)),
    ('bhqd,bhkd->bhqk', (2, 3, 4, 8), (2, 3, 5, 8)),
    ('ij,kj->ik', (4, 6), (5, 6)),
    ('ij,jk', (4, 6), (6, 5)),
    ('abc,cb->a', (3, 4, 5), (5, 4)),
    ('bij,bjk->bki', (2, 3, 4), (2, 4, 5)),
    ('ijk,kl->lji', (2, 3, 4), (4, 5)),
    ('ab,cb->ac', (7, 3), (2, 3)),
    ('xyz,zw->xw', (2, 3, 4), (4, 5)),  # y summed away in x only
])
def test_einsum_lowering_matches_torch(routed, eq, sx, sy):
    g = torch.Generator().manual_seed(0)
    x, y = torch.randn(*sx, generator=g), torch.randn(*sy, generator=g)
    out = hm.einsum(eq, x, y)
    ref = torch.einsum(eq, x, y)
    assert out.shape == ref.shape
    assert torch.allclose(out, ref, atol=1e-5), eq
    assert len(routed) == 1  # one (batched) GEMM per contraction


def test_einsum_falls_back_for_unsupported(routed):
    x = torch.randn(3, 3)
    assert torch.allclose(hm.einsum('ii->i', x), torch.einsum('ii->i', x))
    a, b = torch.randn(2, 3, 4), torch.randn(2, 4, 5)
    assert torch.allclose(hm.einsum('...ij,...jk->...ik', a, b), torch.einsum('...ij,...jk->...ik', a, b))
    assert not routed


def test_bstride_collapse():
    t = torch.zeros(2, 3, 4, 5)
    assert hm._bstride(t, 2) == 20
    e = torch.zeros(1, 3, 4, 5).expand(2, 3, 4, 5)
    assert hm._bstride(e, 2) is None  # [0, 20]: does not collapse to one stride
    b = torch.zeros(4, 5).expand(2, 3, 4, 5)
    assert hm._bstride(b, 2) == 0  # full broadcast
    assert hm._bstride(torch.zeros(1, 1, 4, 5), 2) == 0


def test_matmul_grad_reduction_over_broadcast(routed):
    a = torch.randn(3, 2, 4, 6, requires_grad=True)
    b = torch.randn(2, 6, 5, requires_grad=True)
    y = hm.matmul(a, b)
    (y ** 2).sum().backward()
    a2, b2 = a.detach().clone().requires_grad_(), b.detach().clone().requires_grad_()
    (torch.matmul(a2, b2) ** 2).sum().backward()
    assert torch.allclose(a.grad, a2.grad, atol=1e-4)
    assert torch.allclose(b.grad, b2.grad, atol=1e-4)
    # N-D x 2-D weight: the weight gradient is one flattened GEMM
    x = torch.randn(2, 3, 6, requires_grad=True)
    w = torch.randn(6, 5, requires_grad=True)
    hm.matmul(x, w).sum().backward()
    assert torch.allclose(w.grad, x.detach().reshape(-1, 6).t() @ torch.ones(6, 5))


def test_linear_routes_with_bias_grad(routed, monkeypatch):
    monkeypatch.setattr(hm, '_mm2d', lambda a, b, bias=None, alpha=1.0: (a @ b + (bias if bias is not None else 0)))
    x = torch.randn(4, 3, 8, requires_grad=True)
    w = torch.randn(8, 5, requires_grad=True)
    b = torch.randn(5, requires_grad=True)
    y = hm.linear(x, w, b)
    y.sum().backward()
    assert torch.allclose(y, x @ w + b, atol=1e-5)
    assert torch.allclose(b.grad, torch.full((5,), 12.0))
    assert torch.allclose(w.grad, x.detach().reshape(-1, 8).t() @ torch.ones(12, 5), atol=1e-5)
