"""conv3d depth-tap decomposition (nn/functional/conv.py _conv3d_depth_taps), checked on the CPU with
a torch NHWC conv2d standing in for the HIP kernel: the per-tap depth slices, depth padding,
stride and dilation reproduce torch's conv3d (forward and gradients)."""
import pytest
import torch

import paddle
from paddle.nn.functional import conv as C


def _nhwc_conv2d(x, w, b, s, p, d):
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, b, s, p, d)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize('D,k,s,p,dil', [(8, 3, 1, 1, 1), (9, 3, 2, 1, 1), (10, 3, 1, 2, 2), (7, 1, 1, 0, 1),
                                          (6, 2, 2, 0, 1)])
def test_depth_taps_match_conv3d(monkeypatch, D, k, s, p, dil):
    monkeypatch.setattr(C.ops.conv, 'supported', lambda *a, **kw: True)
    monkeypatch.setattr(C.ops.conv, 'conv2d_nhwc', _nhwc_conv2d)
    torch.manual_seed(D + k)
    x = torch.randn(2, 3, D, 9, 8, dtype=torch.float64, requires_grad=True)
    w = torch.randn(5, 3, k, k, k, dtype=torch.float64, requires_grad=True)
    b = torch.randn(5, dtype=torch.float64, requires_grad=True)
    y = C._conv3d_depth_taps(x, w, b, (s, s, s), (p, p, p), (dil, dil, dil)).permute(0, 4, 1, 2, 3)
    ref = torch.nn.functional.conv3d(x, w, b, s, p, dil)
    assert y.shape == ref.shape
    torch.testing.assert_close(y, ref)
    g = torch.randn_like(ref)
    gx, gw, gb = torch.autograd.grad(y, (x, w, b), g)
    rx, rw, rb = torch.autograd.grad(ref, (x, w, b), g)
    torch.testing.assert_close(gx, rx)
    torch.testing.assert_close(gw, rw)
    torch.testing.assert_close(gb, rb)
