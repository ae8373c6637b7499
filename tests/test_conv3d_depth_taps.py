"""conv3d depth-tap decomposition (nn/functional/conv.py _conv3d_depth_taps), checked on the CPU with
a torch NHWC conv2d standing in for the HIP kernel: the per-tap depth slices, depth padding,
stride and dilation reproduce torch's conv3d (forward and gradients)."""
import pytest
import torch

import paddle
from paddle.nn.functional import conv as C
C_ = C


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


def _nhwc_dwconv2d(x, w, b, s, p, d):
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, b, s, p, d, groups=x.shape[3])
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize('C,Cout,groups,k,s', [(58, 58, 1, 1, 1), (58, 29, 1, 3, 2), (58, 58, 58, 3, 1),
                                                (116, 116, 116, 3, 2)])
def test_cin_padding_matches_conv2d(monkeypatch, C, Cout, groups, k, s):
    """C_in % 8 != 0 (nn/functional/conv.py _conv_cin_pad): zero channels / zero taps on the padded
    channels-last copy reproduce torch's conv2d, forward and gradients (torch convs stand in for the
    HIP kernels)."""
    monkeypatch.setattr(C_.ops.conv, 'supported', lambda x, w, g: x.shape[3] % 8 == 0 and w.shape[0] % 8 == 0)
    monkeypatch.setattr(C_.ops.conv, 'dw_supported', lambda x, w, g: x.shape[3] % 8 == 0)
    monkeypatch.setattr(C_.ops.conv, 'conv2d_nhwc', _nhwc_conv2d)
    monkeypatch.setattr(C_.ops.conv, 'dwconv2d_nhwc', _nhwc_dwconv2d)
    torch.manual_seed(C + k)
    x = torch.randn(2, C, 9, 10, dtype=torch.float64, requires_grad=True)
    w = torch.randn(Cout, C // groups, k, k, dtype=torch.float64, requires_grad=True)
    b = torch.randn(Cout, dtype=torch.float64, requires_grad=True)
    p = k // 2
    y = C_._conv_cin_pad(x, w, b, (s, s), (p, p), (1, 1), groups).permute(0, 3, 1, 2)
    ref = torch.nn.functional.conv2d(x, w, b, s, p, 1, groups)
    torch.testing.assert_close(y, ref)
    g = torch.randn_like(ref)
    for a, r in zip(torch.autograd.grad(y, (x, w, b), g), torch.autograd.grad(ref, (x, w, b), g)):
        torch.testing.assert_close(a, r)


def _nhwc_convt2d(x, w, b, s, p, d, ohw):
    H, W = x.shape[1], x.shape[2]
    op = tuple(ohw[i] - ((x.shape[1 + i] - 1) * s[i] - 2 * p[i] + d[i] * (w.shape[2 + i] - 1) + 1) for i in range(2))
    y = torch.nn.functional.conv_transpose2d(x.permute(0, 3, 1, 2), w, b, s, p, op, 1, d)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize('D,k,s,p,dil,op', [(4, 3, 1, 1, 1, 0), (5, 3, 2, 1, 1, 1), (4, 2, 2, 0, 1, 0), (6, 3, 1, 2, 2, 0)])
def test_convt3d_depth_taps_match_conv_transpose3d(monkeypatch, D, k, s, p, dil, op):
    """conv3d_transpose depth-tap decomposition (_conv_t3d_depth_taps) vs torch conv_transpose3d,
    forward and gradients (torch transposed 2-D convs stand in for the HIP kernels)."""
    monkeypatch.setattr(C.ops.conv, 'convt_supported', lambda *a, **kw: True)
    monkeypatch.setattr(C.ops.conv, 'conv_transpose2d_nhwc', _nhwc_convt2d)
    torch.manual_seed(D * 7 + k)
    x = torch.randn(2, 3, D, 5, 6, dtype=torch.float64, requires_grad=True)
    w = torch.randn(3, 4, k, k, k, dtype=torch.float64, requires_grad=True)
    b = torch.randn(4, dtype=torch.float64, requires_grad=True)
    y = C._conv_t3d_depth_taps(x, w, b, (s, s, s), (p, p, p), (dil, dil, dil), (op, op, op)).permute(0, 4, 1, 2, 3)
    ref = torch.nn.functional.conv_transpose3d(x, w, b, s, p, op, 1, dil)
    assert y.shape == ref.shape
    torch.testing.assert_close(y, ref)
    g = torch.randn_like(ref)
    for a, r in zip(torch.autograd.grad(y, (x, w, b), g), torch.autograd.grad(ref, (x, w, b), g)):
        torch.testing.assert_close(a, r)
