"""Round-5 regression tests (CPU): capture-safe kernel workspaces, weight-only linear autograd."""
import numpy as np
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


def test_update_loss_scaling_zeroes_nonfinite_grads_r6():
    """found_inf zeroes gradients by assignment, so inf / nan entries become 0 too
    (reference FusedFillIf, phi/kernels/gpu/amp_kernel.cu:212)."""
    import paddle
    g = paddle.to_tensor(np.array([1.0, np.inf, np.nan, -2.0], 'float32'))
    found = paddle.to_tensor(np.array([True]))
    sc = paddle.to_tensor(np.array([1024.0], 'float32'))
    good = paddle.to_tensor(np.array([0], 'int32'))
    bad = paddle.to_tensor(np.array([0], 'int32'))
    paddle._C_ops.update_loss_scaling_([g], found, sc, good, bad, 2, 1, 2.0, 0.5)
    np.testing.assert_array_equal(g.numpy(), np.zeros(4, 'float32'))
    assert float(sc) == 512.0
    g2 = paddle.to_tensor(np.array([1.0, 3.0], 'float32'))
    paddle._C_ops.update_loss_scaling_([g2], paddle.to_tensor(np.array([False])), sc, good, bad, 2, 1, 2.0, 0.5)
    np.testing.assert_array_equal(g2.numpy(), np.array([1.0, 3.0], 'float32'))


def test_int4_layout_tag_and_conversion_r6():
    """the int4 packing layout travels with the quantised weight; the old pair layout
    converts losslessly and weight_only_linear converts a tagged old-layout weight."""
    import paddle
    from paddle.nn.quant import quantized_linear as Q
    rs = np.random.RandomState(0)
    w = paddle.to_tensor(rs.randn(16, 8).astype('float32'))
    q, s = Q.weight_quantize(w, algo='weight_only_int4')
    assert q.__dict__['int4_layout'] == Q.INT4_LAYOUT
    old = Q.convert_int4_layout(q, Q.INT4_LAYOUT, 1)
    assert old.__dict__['int4_layout'] == 1
    np.testing.assert_array_equal(Q.convert_int4_layout(old, 1)._t.numpy(), q._t.numpy())
    x = paddle.to_tensor(rs.randn(3, 16).astype('float32'))
    y_new = Q.weight_only_linear(x, q, weight_scale=s, weight_dtype='int4')
    y_old = Q.weight_only_linear(x, old, weight_scale=s, weight_dtype='int4')
    np.testing.assert_allclose(y_old.numpy(), y_new.numpy(), rtol=1e-6)


def test_matmul_autotune_cache_cleared_when_multi_rank_r6(monkeypatch):
    """choices measured before the job became multi-rank are dropped."""
    from paddle.ops import matmul as mm
    mm._TUNE['cache'][('probe',)] = 'lib'
    monkeypatch.setattr(mm, '_multi_rank', lambda: True)
    out = mm._tuned(('other',), lambda: 'hip', lambda: 'lib')
    assert out == 'hip' and ('probe',) not in mm._TUNE['cache']
    mm.clear_tuning()
    assert mm.tuned_choices() == {}


def test_framework_switches_live_in_flags_registry_r6(monkeypatch):
    """The PADDLE_AMD_* A/B switches are FLAGS_pa_* flags (set_flags / FLAGS_ env / legacy env)."""
    import paddle
    from paddle.framework import flags
    assert paddle.get_flags('FLAGS_pa_hip_gemm')['FLAGS_pa_hip_gemm'] is True
    monkeypatch.setenv('PADDLE_AMD_FORCE_COLLECTIVES', '1')
    assert flags.pa_flag('force_collectives') is True
    monkeypatch.setenv('FLAGS_pa_force_collectives', '0')
    assert flags.pa_flag('force_collectives') is False
    old = flags.pa_flag('sot')
    paddle.set_flags({'FLAGS_pa_sot': True})
    try:
        monkeypatch.setenv('PADDLE_AMD_SOT', '0')
        assert flags.pa_flag('sot') is True  # an explicit set_flags wins over the environment
    finally:
        flags._REGISTRY['FLAGS_pa_sot'] = old
        flags._EXPLICIT.discard('FLAGS_pa_sot')
    import os
    import re
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'paddlepaddle-paddle_amd')
    stray = []
    for dp, _, fns in os.walk(root):
        for fn in fns:
            if fn.endswith('.py'):
                for ln in open(os.path.join(dp, fn)):
                    m = re.search(r"os\.environ[^\n]*PADDLE_AMD_([A-Z0-9_]+)", ln)
                    if m and m.group(1) not in ('KERNEL_LIB', 'ARCH'):
                        stray.append((fn, m.group(1)))
    assert not stray, stray
