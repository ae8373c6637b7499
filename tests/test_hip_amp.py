"""csrc/amp.hip: multi-tensor unscale + finite check and the device loss-scale update vs torch."""
import pytest
import torch

pytestmark = pytest.mark.gpu

import paddle  # noqa: E402,F401
from paddle.ops import _native  # noqa: E402
from paddle.ops.amp import check_finite_and_unscale_, update_loss_scaling_  # noqa: E402


def test_check_unscale_mixed_dtypes_many_tensors():
    assert _native._load() is not None
    g = torch.Generator(device='cuda').manual_seed(0)
    sizes = [1, 7, 8, 4093, 65536 + 5, 300000] * 10  # 60 tensors: two launches, tails, odd sizes
    dts = [torch.float32, torch.bfloat16, torch.float16]
    ts = [torch.randn(n, device='cuda', generator=g).to(dts[i % 3]) for i, n in enumerate(sizes)]
    ts.append(torch.randn(33, device='cuda', generator=g)[1:])  # unaligned view
    ref = [t.float() / 4.0 for t in ts]
    found = torch.zeros(1, device='cuda')
    check_finite_and_unscale_(ts, torch.tensor([4.0], device='cuda'), found)
    assert found.item() == 0.0
    for t, r in zip(ts, ref):
        assert torch.allclose(t.float(), r.to(t.dtype).float(), rtol=1e-2, atol=1e-3)
    ts[37][3] = float('inf')
    check_finite_and_unscale_(ts, torch.tensor([1.0], device='cuda'), found)
    assert found.item() == 1.0


def test_update_scale_device():
    sc, gd, bd = (torch.tensor([v], device='cuda') for v in (1024.0, 0.0, 0.0))
    f = torch.ones(1, device='cuda')
    update_loss_scaling_(f, sc, gd, bd, 3, 2, 2.0, 0.5)
    assert sc.item() == 1024.0 and bd.item() == 1.0
    update_loss_scaling_(f, sc, gd, bd, 3, 2, 2.0, 0.5)
    assert sc.item() == 512.0 and bd.item() == 0.0
    f.zero_()
    for _ in range(3):
        update_loss_scaling_(f, sc, gd, bd, 3, 2, 2.0, 0.5)
    assert sc.item() == 1024.0
