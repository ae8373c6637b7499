"""Round-5 regression tests (CPU): capture-safe kernel workspaces, weight-only linear autograd."""
import torch

import paddle
from paddle.ops import workspace as W


def test_workspace_grows_and_retains_captured(monkeypatch):
    ws = W.Workspace('t')
    a = ws.get(100, torch.float32, 'cpu')
    assert a.numel() == 100 and ws.get(50, torch.float32, 'cpu') is a
    b = ws.get(200, torch.float32, 'cpu')  # never captured: the old buffer is dropped
    assert b.numel() == 200 and not ws._retained
    monkeypatch.setattr(torch.cuda, 'is_available', lambda: True)
    monkeypatch.setattr(torch.cuda, 'is_current_stream_capturing', lambda: True)
    assert ws.get(150, torch.float32, 'cpu') is b  # now baked into a "graph"
    monkeypatch.setattr(torch.cuda, 'is_current_stream_capturing', lambda: False)
    c = ws.get(400, torch.float32, 'cpu')
    assert c is not b and ws._retained == [b]  # superseded but still addressed by the graph
    assert ws.release() == 400 * 4 and ws.nbytes() == 200 * 4


def test_workspace_limit():
    ws = W.Workspace('t', limit_bytes=1024)
    assert ws.fits(256, torch.float32) and not ws.fits(257, torch.float32)


def test_weight_only_linear_differentiable_cpu():
    from paddle.nn.quant import weight_quantize, weight_only_linear
    w = torch.randn(64, 32) * 0.1
    q, s = weight_quantize(paddle.to_tensor(w), algo='weight_only_int8')
    x = paddle.randn([3, 64])
    x.stop_gradient = False
    weight_only_linear(x, q, weight_scale=s).sum().backward()
    assert x.grad is not None and x.grad.shape == [3, 64]


def test_c_ops_inplace_fallback_keeps_inplace_semantics():
    x = paddle.to_tensor([1.0, -2.0, 3.0])
    r = paddle._C_ops.hardtanh_(x, -1.0, 1.0)
    assert r is x and x.numpy().tolist() == [1.0, -1.0, 1.0]


def test_amp_loss_scaling_ops_cpu():
    from paddle.ops.amp import check_finite_and_unscale_, update_loss_scaling_
    gs = [torch.tensor([2.0, 4.0]), torch.tensor([1.0, float('nan')], dtype=torch.bfloat16)]
    found = torch.zeros(1)
    check_finite_and_unscale_(gs, torch.tensor([2.0]), found)
    assert gs[0].tolist() == [1.0, 2.0] and found.item() == 1.0
    sc, g, b = torch.tensor([8.0]), torch.zeros(1), torch.zeros(1)
    update_loss_scaling_(found, sc, g, b, 2, 1, 2.0, 0.5)
    assert sc.item() == 4.0
    found.zero_()
    for _ in range(2):
        update_loss_scaling_(found, sc, g, b, 2, 1, 2.0, 0.5)
    assert sc.item() == 8.0 and g.item() == 0.0
