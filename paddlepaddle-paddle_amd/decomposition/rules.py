"""Composite-op decomposition rules (reference: paddle/fluid/primitive/composite/composite.h —
softmax_decomp, log_softmax_decomp, gelu_decomp, silu_decomp, relu/relu6/leaky_relu/elu/hardsigmoid/
hardswish_decomp, layer_norm_decomp, mean_decomp, batch_norm_decomp, group_norm_decomp,
dropout_decomp, square_decomp, reciprocal_decomp, flatten/squeeze/unsqueeze/stack_decomp,
embedding_decomp, clip_decomp).

Each rule takes the recorded node's arguments and rebuilds the op from primitives (elementwise
arithmetic, exp/log/tanh/erf/rsqrt, sum/amax, where/maximum/minimum, matmul, reshape/cat,
index_select).  As in the reference rules, half-precision inputs of the normalisations and softmax
are computed in float32 and cast back.  Reduction counts are ints built from the input's shape (a
SymInt expression of the dynamic dims, evaluated by the Executor at run time).
"""
import math

import torch

from .register import register_decomp

_HALF = (torch.float16, torch.bfloat16)


def _up(x):
    return (x.float(), x.dtype) if x.dtype in _HALF else (x, None)


def _down(y, dt):
    return y.to(dt) if dt is not None else y


def _dims(x, dim):
    if dim is None:
        return list(range(x.dim()))
    if isinstance(dim, int):
        return [dim % max(x.dim(), 1)]
    return [d % x.dim() for d in dim]


def _count(x, dims):
    n = 1
    for d in dims:
        n = n * x.shape[d]  # a SymInt for dynamic dims (static/symbolic.py): no int()
    return n


def _dtype_arg(args, kw):
    dt = kw.get('dtype')
    for a in args:
        if isinstance(a, torch.dtype):
            dt = a
    return dt


@register_decomp('pd_op.softmax')
def softmax(x, dim=None, *args, **kw):
    dt = _dtype_arg(args, kw)
    if dt is not None:
        x = x.to(dt)
    x, back = _up(x)
    d = -1 if dim is None else dim
    e = torch.exp(x - torch.amax(x, d, keepdim=True))
    return _down(e / torch.sum(e, d, keepdim=True), back)


@register_decomp('pd_op.log_softmax')
def log_softmax(x, dim=None, *args, **kw):
    dt = _dtype_arg(args, kw)
    if dt is not None:
        x = x.to(dt)
    x, back = _up(x)
    d = -1 if dim is None else dim
    s = x - torch.amax(x, d, keepdim=True)
    return _down(s - torch.log(torch.sum(torch.exp(s), d, keepdim=True)), back)


@register_decomp('pd_op.gelu')
def gelu(x, approximate='none'):
    x, back = _up(x)
    if approximate == 'tanh':
        inner = math.sqrt(2.0 / math.pi) * (x + 0.044715 * (x * x * x))
        y = 0.5 * x * (1.0 + torch.tanh(inner))
    else:
        y = 0.5 * x * (1.0 + torch.erf(x * (1.0 / math.sqrt(2.0))))
    return _down(y, back)


def _sigmoid(x):
    return 1.0 / (1.0 + torch.exp(-x))


@register_decomp('pd_op.silu')
def silu(x, inplace=False):
    x, back = _up(x)
    return _down(x * _sigmoid(x), back)


@register_decomp('pd_op.relu')
def relu(x, inplace=False):
    return torch.maximum(x, torch.zeros_like(x))


@register_decomp('pd_op.relu6')
def relu6(x, inplace=False):
    return torch.minimum(torch.maximum(x, torch.zeros_like(x)), torch.full_like(x, 6.0))


@register_decomp('pd_op.leaky_relu')
def leaky_relu(x, negative_slope=0.01, inplace=False):
    return torch.where(x > 0, x, x * negative_slope)


@register_decomp('pd_op.elu')
def elu(x, alpha=1.0, inplace=False):
    return torch.where(x > 0, x, alpha * (torch.exp(x) - 1.0))


@register_decomp('pd_op.hardsigmoid')
def hardsigmoid(x, inplace=False):
    return relu6(x + 3.0) / 6.0


@register_decomp('pd_op.hardswish')
def hardswish(x, inplace=False):
    return x * relu6(x + 3.0) / 6.0


@register_decomp('pd_op.layer_norm')
def layer_norm(x, normalized_shape, weight=None, bias=None, eps=1e-5):
    x, back = _up(x)
    nd = len(normalized_shape) if isinstance(normalized_shape, (list, tuple, torch.Size)) else 1
    dims = list(range(x.dim() - nd, x.dim()))
    n = _count(x, dims)
    mean = torch.sum(x, dims, keepdim=True) / n
    xc = x - mean
    var = torch.sum(xc * xc, dims, keepdim=True) / n
    y = xc * torch.rsqrt(var + eps)
    if weight is not None:
        y = y * weight.float()
    if bias is not None:
        y = y + bias.float()
    return _down(y, back)


@register_decomp('pd_op.rms_norm')
def rms_norm(x, normalized_shape, weight=None, eps=None):
    x, back = _up(x)
    nd = len(normalized_shape) if isinstance(normalized_shape, (list, tuple, torch.Size)) else 1
    dims = list(range(x.dim() - nd, x.dim()))
    ms = torch.sum(x * x, dims, keepdim=True) / _count(x, dims)
    y = x * torch.rsqrt(ms + (torch.finfo(x.dtype).eps if eps is None else eps))
    if weight is not None:
        y = y * weight.float()
    return _down(y, back)


@register_decomp('pd_op.mean')
def mean(x, dim=None, keepdim=False, *args, dtype=None, **kw):
    if dtype is not None:
        x = x.to(dtype)
    dims = _dims(x, dim)
    return torch.sum(x, dims, keepdim=keepdim) / _count(x, dims)


@register_decomp('pd_op.addmm')
def addmm(inp, a, b, *, beta=1, alpha=1):
    y = torch.matmul(a, b)
    if alpha != 1:
        y = y * alpha
    return y + (inp * beta if beta != 1 else inp)


@register_decomp('pd_op.linear')
def linear(x, weight, bias=None):
    y = torch.matmul(x, weight.transpose(0, 1))
    return y + bias if bias is not None else y


def _chan_view(t, x):
    return t.reshape([1, -1] + [1] * (x.dim() - 2))


@register_decomp('pd_op.batch_norm')
def batch_norm(x, running_mean, running_var, weight=None, bias=None, training=False, momentum=0.1, eps=1e-5):
    if training:
        raise NotImplementedError("batch_norm: training-mode statistics update is not decomposed")
    x, back = _up(x)
    y = (x - _chan_view(running_mean.float(), x)) * _chan_view(torch.rsqrt(running_var.float() + eps), x)
    if weight is not None:
        y = y * _chan_view(weight.float(), x)
    if bias is not None:
        y = y + _chan_view(bias.float(), x)
    return _down(y, back)


@register_decomp('pd_op.group_norm')
def group_norm(x, num_groups, weight=None, bias=None, eps=1e-5):
    x, back = _up(x)
    shp = list(x.shape)
    g = x.reshape([shp[0], num_groups, -1])
    n = int(g.shape[-1])
    mu = torch.sum(g, [2], keepdim=True) / n
    gc = g - mu
    var = torch.sum(gc * gc, [2], keepdim=True) / n
    y = (gc * torch.rsqrt(var + eps)).reshape(shp)
    if weight is not None:
        y = y * _chan_view(weight.float(), x)
    if bias is not None:
        y = y + _chan_view(bias.float(), x)
    return _down(y, back)


@register_decomp('pd_op.dropout')
def dropout(x, p=0.5, training=True, inplace=False):
    if not training or p == 0.0:
        return x
    if p >= 1.0:
        return x * 0.0
    keep = (torch.rand_like(x, dtype=torch.float32) >= p).to(x.dtype)
    return x * keep * (1.0 / (1.0 - p))


@register_decomp('pd_op.square')
def square(x):
    return x * x


@register_decomp('pd_op.reciprocal')
def reciprocal(x):
    return 1.0 / x


@register_decomp('pd_op.flatten')
def flatten(x, start_dim=0, end_dim=-1):
    nd = x.dim()
    if nd == 0:
        return x.reshape([1])
    s, e = start_dim % nd, end_dim % nd
    shp = list(x.shape)
    n = 1
    for d in range(s, e + 1):
        n *= int(shp[d])
    return x.reshape(shp[:s] + [n] + shp[e + 1:])


@register_decomp('pd_op.squeeze')
def squeeze(x, dim=None):
    shp = list(x.shape)
    if dim is None:
        keep = [s for s in shp if s != 1]
    else:
        ds = {d % max(x.dim(), 1) for d in (dim if isinstance(dim, (list, tuple)) else [dim])}
        keep = [s for i, s in enumerate(shp) if not (i in ds and s == 1)]
    return x.reshape(keep)


@register_decomp('pd_op.unsqueeze')
def unsqueeze(x, dim):
    shp = list(x.shape)
    d = dim % (x.dim() + 1)
    return x.reshape(shp[:d] + [1] + shp[d:])


@register_decomp('pd_op.stack')
def stack(tensors, dim=0):
    return torch.cat([unsqueeze(t, dim) for t in tensors], dim)


@register_decomp('pd_op.embedding')
def embedding(ids, weight, padding_idx=None, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, sparse=False):
    if max_norm is not None:
        raise NotImplementedError("embedding: max_norm renormalisation is not decomposed")
    rows = torch.index_select(weight, 0, ids.reshape([-1]))
    return rows.reshape(list(ids.shape) + [int(weight.shape[1])])


@register_decomp('pd_op.clip')
def clip(x, min=None, max=None):
    y = x
    if min is not None:
        y = torch.where(y < min, torch.full_like(y, float(min)), y)
    if max is not None:
        y = torch.where(y > max, torch.full_like(y, float(max)), y)
    return y
