"""paddle.nn.functional conv / pooling (reference: python/paddle/nn/functional/{conv,pooling}.py).

bf16 2-D convolutions (NCHW or NHWC) run on the hand-written implicit-GEMM kernels of csrc/conv.hip
channels-last; NCHW tensors are carried as NCHW views with channels-last strides, so a default
``data_format='NCHW'`` network pays no layout copies between layers.  Depthwise convolutions run
on csrc/dwconv.hip.  Shapes the kernels reject fall back to the storage layer (MIOpen).
"""
import numpy as np
import torch
import torch.nn.functional as TF

from ... import ops

from ...core.tensor import Tensor, _wrap as _w, _unwrap as _u
from ...tensor._helpers import _shape
from ...core.amp_dispatch import amp_op as _amp_op


def _ntuple(v, n):
    if isinstance(v, Tensor):
        v = v.tolist()
    if isinstance(v, (list, tuple)):
        v = [int(e) for e in v]
        return tuple(v) if len(v) == n else tuple(v * n if len(v) == 1 else v)
    return (int(v),) * n


def _same_pads(in_sz, k, s, d):
    pads = []
    for i, kk, ss, dd in zip(in_sz, k, s, d):
        out = (i + ss - 1) // ss
        tot = max((out - 1) * ss + (kk - 1) * dd + 1 - i, 0)
        pads.append((tot // 2, tot - tot // 2))
    return pads


def _resolve_padding(padding, nd, in_sz=None, k=None, s=None, d=None):
    """Return (torch_padding_tuple, extra_F_pad or None)."""
    if isinstance(padding, str):
        p = padding.upper()
        if p == 'VALID':
            return (0,) * nd, None
        pads = _same_pads(in_sz, k, s, d)
        if all(a == b for a, b in pads):
            return tuple(a for a, _ in pads), None
        flat = []
        for a, b in reversed(pads):
            flat += [a, b]
        return (0,) * nd, flat
    if isinstance(padding, (list, tuple)):
        padding = [(_u(p).item() if isinstance(p, Tensor) else p) for p in padding]
        if len(padding) == nd and all(isinstance(p, int) for p in padding):
            return tuple(padding), None
        if len(padding) == 2 * nd and all(isinstance(p, int) for p in padding):
            pairs = [(padding[2 * i], padding[2 * i + 1]) for i in range(nd)]
            if all(a == b for a, b in pairs):
                return tuple(a for a, _ in pairs), None
            flat = []
            for a, b in reversed(pairs):
                flat += [a, b]
            return (0,) * nd, flat
        if len(padding) == nd + 2:  # [[0,0],[0,0],[a,b],[c,d]] form
            pairs = [tuple(p) for p in padding if isinstance(p, (list, tuple))]
            pairs = pairs[2:] if len(pairs) == nd + 2 else pairs
            if all(a == b for a, b in pairs):
                return tuple(a for a, _ in pairs), None
            flat = []
            for a, b in reversed(pairs):
                flat += [a, b]
            return (0,) * nd, flat
    return _ntuple(padding, nd), None


def _conv(x, weight, bias, stride, padding, dilation, groups, data_format, nd, fn):
    t, w = _u(x), _u(weight)
    b = _u(bias) if bias is not None else None
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, nd + 1, *range(1, nd + 1))
    s, d = _ntuple(stride, nd), _ntuple(dilation, nd)
    p, extra = _resolve_padding(padding, nd, list(t.shape[2:]), list(w.shape[2:]), s, d)
    if extra is not None:
        t = TF.pad(t, extra)
    if nd == 2 and ops.use_hip(t) and ops.conv.supported(t.permute(0, 2, 3, 1), w, groups):
        # conv2d on the hand-written implicit-GEMM kernels (csrc/conv.hip), which run channels-last.
        # NCHW (paddle's default) is served transparently: the NHWC result is returned as an NCHW
        # view with channels-last strides, which the next conv / batch norm / max pool takes
        # without a copy (only a genuinely NCHW-contiguous input, e.g. the image, is repacked once).
        y = ops.conv.conv2d_nhwc(t.permute(0, 2, 3, 1).contiguous(), w, b, s, p, d)
        return _w(y if cl else y.permute(0, 3, 1, 2))
    if nd == 2 and groups == 1 and w.dim() == 4 and w.shape[0] % 8 and ops.use_hip(t):
        # C_out off the 8-channel grain (a 10-class 1x1 head): zero filters pad C_out, the extra
        # output channels are sliced away (their gradients are zero); autograd maps the padded
        # filter / bias gradients back
        cp = -(-w.shape[0] // 8) * 8 - w.shape[0]
        wp = TF.pad(w, (0, 0, 0, 0, 0, 0, 0, cp))
        if ops.conv.supported(t.permute(0, 2, 3, 1), wp, 1):
            bp = None if b is None else TF.pad(b, (0, cp))
            y = ops.conv.conv2d_nhwc(t.permute(0, 2, 3, 1).contiguous(), wp, bp, s, p, d)[..., :w.shape[0]]
            y = y.contiguous()
            return _w(y if cl else y.permute(0, 3, 1, 2))
    if (nd == 2 and w.dim() == 4 and t.shape[1] >= 8 and t.shape[1] % 8 and (groups == 1 or groups == t.shape[1])
            and ops.use_hip(t)):
        # C_in off the 8-channel grain (ShuffleNet's 58 / 116-channel branches): the channels-last
        # input is zero-padded to the grain (one copy) with zero filter taps for the extra channels
        # (plain conv: extra input channels; depthwise: extra channels sliced off the output)
        y = _conv_cin_pad(t, w, b, s, p, d, groups)
        if y is not None:
            return _w(y if cl else y.permute(0, 3, 1, 2))
    if nd == 3 and groups == 1 and ops.use_hip(t) and w.dim() == 5:
        y = _conv3d_depth_taps(t, w, b, s, p, d)
        if y is not None:
            return _w(y if cl else y.permute(0, 4, 1, 2, 3))
    if nd == 2 and ops.use_hip(t) and ops.conv.dw_supported(t.permute(0, 2, 3, 1), w, groups):
        # depthwise (groups == C_in == C_out) on csrc/dwconv.hip, channels-last as above
        y = ops.conv.dwconv2d_nhwc(t.permute(0, 2, 3, 1).contiguous(), w, b, s, p, d)
        return _w(y if cl else y.permute(0, 3, 1, 2))
    if nd == 2 and ops.use_hip(t) and ops.conv.gconv_supported(t.permute(0, 2, 3, 1), w, groups, s, p, d):
        # grouped (1 < groups < C_in: ResNeXt) on csrc/gconv.hip, channels-last as above
        y = ops.conv.gconv2d_nhwc(t.permute(0, 2, 3, 1).contiguous(), w, b, groups, s, p, d)
        return _w(y if cl else y.permute(0, 3, 1, 2))
    out = fn(t, w, b, s, p, d, groups)
    if cl:
        out = out.permute(0, *range(2, nd + 2), 1)
    return _w(out)


def _conv_cin_pad(t, w, b, s, p, d, groups):
    """conv2d / depthwise conv2d of an NCHW(-viewed) t whose channel count C is not a multiple of 8,
    on the hand-written channels-last kernels over a zero-padded copy; returns NHWC or None."""
    C = t.shape[1]
    cp = -(-C // 8) * 8 - C
    xp = TF.pad(t.permute(0, 2, 3, 1), (0, cp))                     # NHWC, channels padded, contiguous
    if groups == 1:
        co = w.shape[0]
        cop = -(-co // 8) * 8 - co
        wp = TF.pad(w, (0, 0, 0, 0, 0, cp, 0, cop))                  # zero taps: extra in / out channels
        bp = None if b is None else TF.pad(b, (0, cop))
        if not ops.conv.supported(xp, wp, 1):
            return None
        y = ops.conv.conv2d_nhwc(xp, wp, bp, s, p, d)
        return y[..., :co].contiguous() if cop else y
    wp = TF.pad(w, (0, 0, 0, 0, 0, 0, 0, cp))                        # [C + cp, 1, R, S]
    bp = None if b is None else TF.pad(b, (0, cp))
    if not ops.conv.dw_supported(xp, wp, C + cp):
        return None
    return ops.conv.dwconv2d_nhwc(xp, wp, bp, s, p, d)[..., :C].contiguous()


def _conv3d_depth_taps(t, w, b, s, p, d):
    """conv3d on the 2-D implicit-GEMM kernels: for every depth tap z of the filter, the input depth
    slices that tap reads (stride s[0], dilation d[0], zero depth padding p[0]) are folded into the
    batch — [N * D_out, H, W, C] channels-last — and convolved with the tap's 2-D filter w[:, :, z];
    the kd partial outputs add up.  Differentiable through the 2-D kernels' backward.  Returns the
    NDHWC output, or None when a 2-D sub-problem is outside the kernels' contract."""
    N, C, D, H, W = t.shape
    kd = w.shape[2]
    Do = (D + 2 * p[0] - d[0] * (kd - 1) - 1) // s[0] + 1
    if Do <= 0:
        return None
    xn = t.permute(0, 2, 3, 4, 1)  # NDHWC view
    if p[0]:
        xn = TF.pad(xn, (0, 0, 0, 0, 0, 0, p[0], p[0]))
    y = None
    for z in range(kd):
        lo = z * d[0]
        xz = xn[:, lo:lo + (Do - 1) * s[0] + 1:s[0]].reshape(N * Do, H, W, C)
        wz = w[:, :, z]
        if not ops.conv.supported(xz, wz, 1):
            return None
        yz = ops.conv.conv2d_nhwc(xz.contiguous(), wz.contiguous(), b if z == 0 else None, s[1:], p[1:], d[1:])
        y = yz if y is None else y + yz
    return y.reshape(N, Do, y.shape[1], y.shape[2], y.shape[3])


@_amp_op('conv2d')
def conv1d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format='NCL', name=None):
    t, w = _u(x), _u(weight)
    if ops.use_hip(t) and t.dim() == 3 and w.dim() == 3 and not isinstance(padding, str) and groups == 1:
        # a 1-D convolution is a 2-D one over a height-1 image: the channels-last HIP kernels
        cl = data_format[-1] == 'C'
        xn = (t if cl else t.permute(0, 2, 1)).unsqueeze(1)  # [N, 1, L, C]
        w4 = w.unsqueeze(2)
        pd = _ntuple(padding, 1)
        if len(pd) == 1 and ops.conv.supported(xn, w4, 1):
            y = ops.conv.conv2d_nhwc(xn.contiguous(), w4, None if bias is None else _u(bias), (1, _ntuple(stride, 1)[0]),
                                     (0, pd[0]), (1, _ntuple(dilation, 1)[0]))[:, 0]  # [N, Lo, Cout]
            return _w(y if cl else y.permute(0, 2, 1))
    return _conv(x, weight, bias, stride, padding, dilation, groups, data_format, 1, TF.conv1d)


@_amp_op('conv2d')
def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format='NCHW', name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, data_format, 2, TF.conv2d)


@_amp_op('conv3d')
def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format='NCDHW', name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, data_format, 3, TF.conv3d)


def _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, output_size, data_format, nd, fn):
    t, w = _u(x), _u(weight)
    b = _u(bias) if bias is not None else None
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, nd + 1, *range(1, nd + 1))
    s, d = _ntuple(stride, nd), _ntuple(dilation, nd)
    if isinstance(padding, str):
        p = (0,) * nd if padding.upper() == 'VALID' else tuple(((w.shape[2 + i] - 1) * d[i]) // 2 for i in range(nd))
    else:
        p, _ = _resolve_padding(padding, nd)
    op = _ntuple(output_padding, nd)
    if output_size is not None:
        osz = _ntuple(output_size, nd) if not isinstance(output_size, int) else (output_size,) * nd
        op = tuple(osz[i] - ((t.shape[2 + i] - 1) * s[i] - 2 * p[i] + d[i] * (w.shape[2 + i] - 1) + 1) for i in range(nd))
    if nd == 2 and ops.use_hip(t):
        ohw = tuple((t.shape[2 + i] - 1) * s[i] - 2 * p[i] + d[i] * (w.shape[2 + i] - 1) + op[i] + 1 for i in range(2))
        xn = t.permute(0, 2, 3, 1)
        if ops.conv.convt_supported(xn, w, groups, s, p, d, ohw):
            # transposed conv on the stride-class data-gradient kernel (channels-last, NCHW as views)
            y = ops.conv.conv_transpose2d_nhwc(xn.contiguous(), w, b, s, p, d, ohw)
            return _w(y if cl else y.permute(0, 3, 1, 2))
    if nd == 3 and groups == 1 and ops.use_hip(t) and w.dim() == 5:
        y = _conv_t3d_depth_taps(t, w, b, s, p, d, op)
        if y is not None:
            return _w(y if cl else y.permute(0, 4, 1, 2, 3))
    out = fn(t, w, b, s, p, op, groups, d)
    if cl:
        out = out.permute(0, *range(2, nd + 2), 1)
    return _w(out)


def _conv_t3d_depth_taps(t, w, b, s, p, d, op):
    """conv3d_transpose on the 2-D transposed-conv kernels: every depth tap z of the filter is one
    batched 2-D transposed convolution of all input depth slices (folded into the batch, channels
    last) with the tap's 2-D filter w[:, :, z]; input slice i lands on output depth
    i * s[0] - p[0] + z * d[0] (index_add, slices outside [0, D_out) dropped).  Differentiable
    through the 2-D kernels' backward.  Returns NDHWC, or None outside the kernels' contract."""
    N, C, D, H, W = t.shape
    kd = w.shape[2]
    Do = (D - 1) * s[0] - 2 * p[0] + d[0] * (kd - 1) + op[0] + 1
    ohw = tuple((t.shape[3 + i] - 1) * s[1 + i] - 2 * p[1 + i] + d[1 + i] * (w.shape[3 + i] - 1) + op[1 + i] + 1
                for i in range(2))
    if Do <= 0 or min(ohw) <= 0:
        return None
    xn = t.permute(0, 2, 3, 4, 1).reshape(N * D, H, W, C)
    if not ops.conv.convt_supported(xn, w[:, :, 0], 1, s[1:], p[1:], d[1:], ohw):
        return None
    xn = xn.contiguous()
    y = None
    src = torch.arange(D, device=t.device)
    for z in range(kd):
        dst = src * s[0] - p[0] + z * d[0]
        keep = (dst >= 0) & (dst < Do)
        if not bool(keep.any()):
            continue
        yz = ops.conv.conv_transpose2d_nhwc(xn, w[:, :, z].contiguous(), None, s[1:], p[1:], d[1:], ohw)
        yz = yz.reshape(N, D, ohw[0], ohw[1], -1)
        if y is None:
            y = yz.new_zeros(N, Do, ohw[0], ohw[1], yz.shape[-1])
        y = y.index_add(1, dst[keep], yz[:, keep])
    if y is None:
        return None
    if b is not None:
        y = y + b.to(y.dtype)
    return y


def conv1d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format='NCL', name=None):
    return _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, output_size, data_format, 1,
                   TF.conv_transpose1d)


def conv2d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, dilation=1, groups=1,
                     output_size=None, data_format='NCHW', name=None):
    return _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, output_size, data_format, 2,
                   TF.conv_transpose2d)


def conv3d_transpose(x, weight, bias=None, stride=1, padding=0, output_padding=0, groups=1, dilation=1,
                     output_size=None, data_format='NCDHW', name=None):
    return _conv_t(x, weight, bias, stride, padding, output_padding, dilation, groups, output_size, data_format, 3,
                   TF.conv_transpose3d)


# ----------------------------------------------------------------------------- pooling
def _pool(x, kernel_size, stride, padding, ceil_mode, data_format, nd, fn, extra=None, return_mask=False):
    t = _u(x)
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, nd + 1, *range(1, nd + 1))
    k = _ntuple(kernel_size, nd)
    s = k if stride is None else _ntuple(stride, nd)
    p, pre = _resolve_padding(padding, nd, list(t.shape[2:]), k, s, (1,) * nd)
    if pre is not None:
        t = TF.pad(t, pre, value=float('-inf') if fn in (TF.max_pool1d, TF.max_pool2d, TF.max_pool3d) else 0.0)
    kw = dict(extra or {})
    if nd == 2 and fn is TF.max_pool2d and not return_mask and pre is None and ops.use_hip(t):
        # NHWC max pool on csrc/pool.hip (one-byte argmax, atomics-free gather backward); an NCHW
        # tensor with channels-last strides (the output of a routed conv2d) is the same memory
        xn = _u(x) if cl else t.permute(0, 2, 3, 1)
        if (cl or xn.is_contiguous()) and ops.pool.supported(xn, k, s, p):
            y = ops.pool.max_pool2d_nhwc(xn, k, s, p, ceil_mode)
            return _w(y if cl else y.permute(0, 3, 1, 2))
    if return_mask:
        out, mask = fn(t, k, s, p, ceil_mode=ceil_mode, return_indices=True, **kw)
        if cl:
            out = out.permute(0, *range(2, nd + 2), 1)
            mask = mask.permute(0, *range(2, nd + 2), 1)
        return _w(out), _w(mask)
    out = fn(t, k, s, p, ceil_mode=ceil_mode, **kw)
    if cl:
        out = out.permute(0, *range(2, nd + 2), 1)
    return _w(out)


def max_pool1d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, 'NCL', 1, TF.max_pool1d, return_mask=return_mask)


@_amp_op('max_pool2d_with_index')
def max_pool2d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format='NCHW',
               name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 2, TF.max_pool2d, return_mask=return_mask)


def max_pool3d(x, kernel_size, stride=None, padding=0, return_mask=False, ceil_mode=False, data_format='NCDHW',
               name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 3, TF.max_pool3d, return_mask=return_mask)


def avg_pool1d(x, kernel_size, stride=None, padding=0, exclusive=True, ceil_mode=False, name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, 'NCL', 1, TF.avg_pool1d,
                 {'count_include_pad': not exclusive})


def avg_pool2d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format='NCHW', name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 2, TF.avg_pool2d,
                 {'count_include_pad': not exclusive, 'divisor_override': divisor_override})


def avg_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, exclusive=True, divisor_override=None,
               data_format='NCDHW', name=None):
    return _pool(x, kernel_size, stride, padding, ceil_mode, data_format, 3, TF.avg_pool3d,
                 {'count_include_pad': not exclusive, 'divisor_override': divisor_override})


def lp_pool1d(x, norm_type, kernel_size, stride=None, ceil_mode=False, data_format='NCL', name=None):
    return _w(TF.lp_pool1d(_u(x), norm_type, kernel_size, stride, ceil_mode))


def lp_pool2d(x, norm_type, kernel_size, stride=None, ceil_mode=False, data_format='NCHW', name=None):
    return _w(TF.lp_pool2d(_u(x), norm_type, kernel_size, stride, ceil_mode))


def _adaptive(x, output_size, data_format, nd, fn, return_mask=False):
    t = _u(x)
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, nd + 1, *range(1, nd + 1))
    if isinstance(output_size, (list, tuple)):
        output_size = tuple(t.shape[2 + i] if o is None else int(o) for i, o in enumerate(output_size))
    if return_mask:
        out, m = fn(t, output_size, return_indices=True)
        if cl:
            out, m = out.permute(0, *range(2, nd + 2), 1), m.permute(0, *range(2, nd + 2), 1)
        return _w(out), _w(m)
    out = fn(t, output_size)
    if cl:
        out = out.permute(0, *range(2, nd + 2), 1)
    return _w(out)


def adaptive_avg_pool1d(x, output_size, name=None):
    return _adaptive(x, output_size, 'NCL', 1, TF.adaptive_avg_pool1d)


def adaptive_avg_pool2d(x, output_size, data_format='NCHW', name=None):
    return _adaptive(x, output_size, data_format, 2, TF.adaptive_avg_pool2d)


def adaptive_avg_pool3d(x, output_size, data_format='NCDHW', name=None):
    return _adaptive(x, output_size, data_format, 3, TF.adaptive_avg_pool3d)


def adaptive_max_pool1d(x, output_size, return_mask=False, name=None):
    return _adaptive(x, output_size, 'NCL', 1, TF.adaptive_max_pool1d, return_mask)


def adaptive_max_pool2d(x, output_size, return_mask=False, name=None):
    return _adaptive(x, output_size, 'NCHW', 2, TF.adaptive_max_pool2d, return_mask)


def adaptive_max_pool3d(x, output_size, return_mask=False, name=None):
    return _adaptive(x, output_size, 'NCDHW', 3, TF.adaptive_max_pool3d, return_mask)


def _unpool(x, indices, kernel_size, stride, padding, output_size, nd, fn, data_format):
    k = _ntuple(kernel_size, nd)
    s = k if stride is None else _ntuple(stride, nd)
    p = _ntuple(padding, nd)
    return _w(fn(_u(x), _u(indices), k, s, p, output_size))


def max_unpool1d(x, indices, kernel_size, stride=None, padding=0, data_format='NCL', output_size=None, name=None):
    return _unpool(x, indices, kernel_size, stride, padding, output_size, 1, TF.max_unpool1d, data_format)


def max_unpool2d(x, indices, kernel_size, stride=None, padding=0, data_format='NCHW', output_size=None, name=None):
    return _unpool(x, indices, kernel_size, stride, padding, output_size, 2, TF.max_unpool2d, data_format)


def max_unpool3d(x, indices, kernel_size, stride=None, padding=0, data_format='NCDHW', output_size=None, name=None):
    return _unpool(x, indices, kernel_size, stride, padding, output_size, 3, TF.max_unpool3d, data_format)


def fractional_max_pool2d(x, output_size, kernel_size=None, random_u=None, return_mask=False, name=None):
    k = kernel_size or 2
    r = TF.fractional_max_pool2d(_u(x), k, output_size=output_size, return_indices=return_mask)
    return (_w(r[0]), _w(r[1])) if return_mask else _w(r)


def fractional_max_pool3d(x, output_size, kernel_size=None, random_u=None, return_mask=False, name=None):
    k = kernel_size or 2
    r = TF.fractional_max_pool3d(_u(x), k, output_size=output_size, return_indices=return_mask)
    return (_w(r[0]), _w(r[1])) if return_mask else _w(r)
