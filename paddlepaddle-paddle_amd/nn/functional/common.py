"""paddle.nn.functional common ops (reference: python/paddle/nn/functional/{common,input,vision,distance,extension}.py)."""
import math

import numpy as np
import torch
import torch.nn.functional as TF

from ...core.tensor import Tensor, _wrap as _w, _unwrap as _u
from ...core import dtype as _dt
from ...tensor._helpers import _shape
from ... import ops
from ...core.amp_dispatch import amp_op as _amp_op


_ZB = [None]  # distributed.fleet.meta_parallel.zero_bubble_utils, imported on first use


@_amp_op('matmul_v2')
def linear(x, weight, bias=None, name=None):
    """y = x @ W + b with W stored [in_features, out_features] (paddle layout)."""
    t, w = _u(x), _u(weight)
    b = _u(bias) if bias is not None else None
    if _ZB[0] is None:
        from ...distributed.fleet.meta_parallel import zero_bubble_utils as _zbm
        _ZB[0] = _zbm
    if _ZB[0].WeightGradStore.active and w.requires_grad and torch.is_grad_enabled():
        return _w(_ZB[0].split_linear(t, w, b, weight, bias))  # zero-bubble pipeline: dW deferred to W
    if ops.fp8._ACTIVE['enabled'] and ops.fp8.eligible(t, w):  # paddle.amp.fp8_autocast
        return _w(ops.fp8.fp8_linear(t, w, b, holder=weight if isinstance(weight, Tensor) else None))
    if isinstance(weight, Tensor) and '_flat' in weight.__dict__ and ops.linear.eligible(weight) and \
            (bias is None or '_flat' in bias.__dict__):
        return _w(ops.linear.linear_accum(t, weight, bias))
    # everything else (eval / no_grad / inference, weights outside flat buffers): all three GEMMs on
    # the hand-written kernel for bf16 / fp16 GPU operands (ops/matmul.py), else torch
    return _w(ops.matmul.linear(t, w, b))


def bilinear(x1, x2, weight, bias=None, name=None):
    return _w(TF.bilinear(_u(x1), _u(x2), _u(weight), None if bias is None else _u(bias).reshape(-1)))


def dropout(x, p=0.5, axis=None, training=True, mode='upscale_in_train', name=None):
    t = _u(x)
    if not training or p == 0:
        if mode == 'downscale_in_infer' and not training:
            return _w(t * (1.0 - p))
        return x if isinstance(x, Tensor) else _w(t)
    if p == 1:
        return _w(torch.zeros_like(t))
    if axis is not None:
        axes = [axis] if isinstance(axis, int) else list(axis)
        mshape = [s if i in axes or i - t.dim() in axes else 1 for i, s in enumerate(t.shape)]
        mask = (torch.rand(mshape, device=t.device) >= p).to(t.dtype)
        return _w(t * mask / (1 - p) if mode == 'upscale_in_train' else t * mask)
    if mode == 'upscale_in_train':
        if ops.use_hip(t) and t.is_contiguous():
            return _w(ops.act.dropout(t, p))
        return _w(TF.dropout(t, p, True))
    mask = (torch.rand_like(t, dtype=torch.float32) >= p).to(t.dtype)
    return _w(t * mask)


def dropout2d(x, p=0.5, training=True, data_format='NCHW', name=None):
    t = _u(x)
    if data_format == 'NHWC':
        return _w(TF.dropout2d(t.permute(0, 3, 1, 2), p, training).permute(0, 2, 3, 1))
    return _w(TF.dropout2d(t, p, training))


def dropout3d(x, p=0.5, training=True, data_format='NCDHW', name=None):
    t = _u(x)
    if data_format == 'NDHWC':
        return _w(TF.dropout3d(t.permute(0, 4, 1, 2, 3), p, training).permute(0, 2, 3, 4, 1))
    return _w(TF.dropout3d(t, p, training))


def alpha_dropout(x, p=0.5, training=True, name=None):
    return _w(TF.alpha_dropout(_u(x), p, training))


def feature_alpha_dropout(x, p=0.5, training=True, name=None):
    return _w(TF.feature_alpha_dropout(_u(x), p, training))


def _pad_list(pad, nd, data_format):
    """paddle pad list is ordered from the FIRST spatial dim; torch from the LAST."""
    pad = _shape(pad)
    if len(pad) == 2 * nd:
        pairs = [pad[i:i + 2] for i in range(0, len(pad), 2)]
        return [v for pr in reversed(pairs) for v in pr]
    return pad


def pad(x, pad, mode='constant', value=0.0, data_format='NCHW', pad_from_left_axis=True, name=None):
    t = _u(x)
    p = _shape(pad)
    nd = t.dim()
    if len(p) == 2 * nd:  # full-rank paddle pad: [d0_lo, d0_hi, d1_lo, ...]
        pairs = [p[i:i + 2] for i in range(0, len(p), 2)]
        tp = [v for pr in reversed(pairs) for v in pr]
        if mode == 'constant':
            return _w(TF.pad(t, tp, 'constant', value))
        return _w(TF.pad(t, tp[:2 * (nd - 2)], mode if mode != 'edge' else 'replicate'))
    channel_last = data_format[-1] == 'C'
    if channel_last:
        perm = [0, nd - 1] + list(range(1, nd - 1))
        t = t.permute(*perm)
    # spatial pads given as [left, right, top, bottom, ...] (last dim first, paddle 4-D convention)
    m = {'constant': 'constant', 'reflect': 'reflect', 'replicate': 'replicate', 'edge': 'replicate',
         'circular': 'circular'}[mode]
    out = TF.pad(t, p, m, value) if m == 'constant' else TF.pad(t, p, m)
    if channel_last:
        inv = [0] + list(range(2, nd)) + [1]
        out = out.permute(*inv)
    return _w(out)


def zeropad2d(x, padding, data_format='NCHW', name=None):
    return pad(x, padding, 'constant', 0.0, data_format)


@_amp_op('bilinear_interp_v2')
def interpolate(x, size=None, scale_factor=None, mode='nearest', align_corners=False, align_mode=0,
                data_format=None, recompute_scale_factor=None, name=None):
    t = _u(x)
    nd = t.dim()
    data_format = data_format or {3: 'NCW', 4: 'NCHW', 5: 'NCDHW'}[nd]
    cl = data_format[-1] == 'C'
    if cl:
        t = t.permute(0, nd - 1, *range(1, nd - 1))
    if size is not None:
        size = _shape(size) if not isinstance(size, int) else size
    if isinstance(scale_factor, Tensor):
        scale_factor = scale_factor.tolist()
    m = {'nearest': 'nearest', 'bilinear': 'bilinear', 'trilinear': 'trilinear', 'bicubic': 'bicubic',
         'linear': 'linear', 'area': 'area'}[mode.lower()]
    kw = {}
    if m in ('bilinear', 'trilinear', 'bicubic', 'linear'):
        kw['align_corners'] = align_corners
    out = TF.interpolate(t, size=size, scale_factor=scale_factor, mode=m, **kw)
    if cl:
        out = out.permute(0, *range(2, nd), 1)
    return _w(out)


upsample = interpolate


@_amp_op('lookup_table_v2')
def embedding(x, weight, padding_idx=None, max_norm=None, norm_type=2.0, sparse=False, scale_grad_by_freq=False,
              name=None):
    ids, w = _u(x), _u(weight)
    if padding_idx is not None and padding_idx < 0:
        padding_idx += w.shape[0]
    if ops.use_hip(w) and ops.use_hip(ids) and max_norm is None:
        return _w(ops.embedding.embedding(ids, w, padding_idx))
    return _w(TF.embedding(ids, w, padding_idx, max_norm, norm_type, scale_grad_by_freq, sparse))


def one_hot(x, num_classes, name=None):
    return _w(TF.one_hot(_u(x).long(), num_classes).to(torch.float32))


def label_smooth(label, prior_dist=None, epsilon=0.1, name=None):
    t = _u(label)
    if prior_dist is not None:
        return _w((1 - epsilon) * t + epsilon * _u(prior_dist))
    return _w((1 - epsilon) * t + epsilon / t.shape[-1])


def sequence_mask(x, maxlen=None, dtype='int64', name=None):
    t = _u(x)
    m = int(t.max().item()) if maxlen is None else int(maxlen._t.item() if isinstance(maxlen, Tensor) else maxlen)
    r = torch.arange(m, device=t.device)
    return _w((r < t.unsqueeze(-1)).to(_dt.to_torch_dtype(dtype)))


def cosine_similarity(x1, x2, axis=1, eps=1e-8):
    return _w(TF.cosine_similarity(_u(x1), _u(x2), axis, eps))


def pairwise_distance(x, y, p=2.0, epsilon=1e-6, keepdim=False, name=None):
    return _w(TF.pairwise_distance(_u(x), _u(y), p, epsilon, keepdim))


def normalize(x, p=2, axis=1, epsilon=1e-12, name=None):
    return _w(TF.normalize(_u(x), p, axis, epsilon))


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    p = paddings
    if isinstance(p, (list, tuple)) and len(p) == 4:
        t = TF.pad(_u(x), [p[1], p[3], p[0], p[2]])
        return _w(TF.unfold(t, kernel_sizes, dilations, 0, strides))
    return _w(TF.unfold(_u(x), kernel_sizes, dilations, p, strides))


def fold(x, output_sizes, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return _w(TF.fold(_u(x), output_sizes, kernel_sizes, dilations, paddings, strides))


def pixel_shuffle(x, upscale_factor, data_format='NCHW', name=None):
    t = _u(x)
    if data_format == 'NHWC':
        return _w(TF.pixel_shuffle(t.permute(0, 3, 1, 2), upscale_factor).permute(0, 2, 3, 1))
    return _w(TF.pixel_shuffle(t, upscale_factor))


def pixel_unshuffle(x, downscale_factor, data_format='NCHW', name=None):
    t = _u(x)
    if data_format == 'NHWC':
        return _w(TF.pixel_unshuffle(t.permute(0, 3, 1, 2), downscale_factor).permute(0, 2, 3, 1))
    return _w(TF.pixel_unshuffle(t, downscale_factor))


def channel_shuffle(x, groups, data_format='NCHW', name=None):
    t = _u(x)
    if data_format == 'NHWC':
        return _w(TF.channel_shuffle(t.permute(0, 3, 1, 2), groups).permute(0, 2, 3, 1))
    return _w(TF.channel_shuffle(t, groups))


def affine_grid(theta, out_shape, align_corners=True, name=None):
    return _w(TF.affine_grid(_u(theta), _shape(out_shape), align_corners=align_corners))


def grid_sample(x, grid, mode='bilinear', padding_mode='zeros', align_corners=True, name=None):
    return _w(TF.grid_sample(_u(x), _u(grid), mode, padding_mode, align_corners))


def temporal_shift(x, seg_num, shift_ratio=0.25, name=None, data_format='NCHW'):
    t = _u(x)
    if data_format == 'NHWC':
        t = t.permute(0, 3, 1, 2)
    nt, c, h, w = t.shape
    t5 = t.reshape(nt // seg_num, seg_num, c, h, w)
    c1 = int(c * shift_ratio)
    c2 = int(c * 2 * shift_ratio)
    out = torch.zeros_like(t5)
    out[:, :-1, :c1] = t5[:, 1:, :c1]
    out[:, 1:, c1:c2] = t5[:, :-1, c1:c2]
    out[:, :, c2:] = t5[:, :, c2:]
    out = out.reshape(nt, c, h, w)
    if data_format == 'NHWC':
        out = out.permute(0, 2, 3, 1)
    return _w(out)


def class_center_sample(label, num_classes, num_samples, group=None):
    t = _u(label)
    pos = torch.unique(t)
    if pos.numel() < num_samples:
        neg = torch.tensor([c for c in range(num_classes) if c not in set(pos.tolist())], device=t.device)
        neg = neg[torch.randperm(neg.numel(), device=t.device)[:num_samples - pos.numel()]]
        sampled = torch.sort(torch.cat([pos, neg]))[0]
    else:
        sampled = pos
    remap = torch.full((num_classes,), -1, dtype=torch.long, device=t.device)
    remap[sampled] = torch.arange(sampled.numel(), device=t.device)
    return _w(remap[t]), _w(sampled)


def gather_tree(ids, parents):
    i, p = _u(ids), _u(parents)
    T = i.shape[0]
    out = torch.empty_like(i)
    out[-1] = i[-1]
    par = p[-1]
    for step in range(T - 2, -1, -1):
        out[step] = torch.gather(i[step], -1, par)
        par = torch.gather(p[step], -1, par)
    return _w(out)


def diag_embed(input, offset=0, dim1=-2, dim2=-1):  # noqa: A002
    return _w(torch.diag_embed(_u(input), offset, dim1, dim2))
