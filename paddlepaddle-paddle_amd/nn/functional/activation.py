"""paddle.nn.functional activations (reference: python/paddle/nn/functional/activation.py).

gelu / silu / swiglu / softmax on HIP tensors route to the hand-written kernels in
``ops/`` (fused, vectorised bf16); everything else maps onto the storage layer.
"""
import torch
import torch.nn.functional as TF

from ...core.tensor import Tensor, _wrap as _w, _unwrap as _u
from ...core import dtype as _dt
from ... import ops
from ...core.amp_dispatch import amp_op as _amp_op


def relu(x, name=None):
    return _w(torch.relu(_u(x)))


def relu_(x, name=None):
    x._t.relu_()
    return x


def relu6(x, name=None):
    return _w(TF.relu6(_u(x)))


def leaky_relu(x, negative_slope=0.01, name=None):
    return _w(TF.leaky_relu(_u(x), negative_slope))


def leaky_relu_(x, negative_slope=0.01, name=None):
    TF.leaky_relu_(x._t, negative_slope)
    return x


def elu(x, alpha=1.0, name=None):
    return _w(TF.elu(_u(x), alpha))


def elu_(x, alpha=1.0, name=None):
    TF.elu_(x._t, alpha)
    return x


def celu(x, alpha=1.0, name=None):
    return _w(TF.celu(_u(x), alpha))


def selu(x, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717, name=None):
    t = _u(x)
    return _w(scale * torch.where(t > 0, t, alpha * (torch.exp(t) - 1)))


def gelu(x, approximate=False, name=None):
    t = _u(x)
    if ops.use_hip(t):
        return _w(ops.act.gelu(t, approximate))
    return _w(TF.gelu(t, approximate='tanh' if approximate else 'none'))


def silu(x, name=None):
    t = _u(x)
    if ops.use_hip(t):
        return _w(ops.act.silu(t))
    return _w(TF.silu(t))


def swish(x, name=None):
    return silu(x)


def mish(x, name=None):
    return _w(TF.mish(_u(x)))


def sigmoid(x, name=None):
    return _w(torch.sigmoid(_u(x)))


def hardsigmoid(x, slope=0.1666667, offset=0.5, name=None):
    t = _u(x)
    return _w(torch.clamp(t * slope + offset, 0.0, 1.0))


def hardswish(x, name=None):
    return _w(TF.hardswish(_u(x)))


def hardtanh(x, min=-1.0, max=1.0, name=None):  # noqa: A002
    return _w(TF.hardtanh(_u(x), min, max))


def hardtanh_(x, min=-1.0, max=1.0, name=None):  # noqa: A002
    TF.hardtanh_(x._t, min, max)
    return x


def hardshrink(x, threshold=0.5, name=None):
    return _w(TF.hardshrink(_u(x), threshold))


def softshrink(x, threshold=0.5, name=None):
    return _w(TF.softshrink(_u(x), threshold))


@_amp_op('tanh_shrink')
def tanhshrink(x, name=None):
    return _w(TF.tanhshrink(_u(x)))


def softsign(x, name=None):
    return _w(TF.softsign(_u(x)))


@_amp_op('softplus')
def softplus(x, beta=1, threshold=20, name=None):
    return _w(TF.softplus(_u(x), beta, threshold))


def log_sigmoid(x, name=None):
    return _w(TF.logsigmoid(_u(x)))


def tanh(x, name=None):
    return _w(torch.tanh(_u(x)))


def tanh_(x, name=None):
    x._t.tanh_()
    return x


def thresholded_relu(x, threshold=1.0, value=0.0, name=None):
    t = _u(x)
    return _w(torch.where(t > threshold, t, torch.full_like(t, value)))


def thresholded_relu_(x, threshold=1.0, value=0.0, name=None):
    x._t.copy_(thresholded_relu(x, threshold, value)._t)
    return x


def prelu(x, weight, data_format='NCHW', name=None):
    t, w = _u(x), _u(weight)
    if w.numel() > 1 and data_format[-1] == 'C' and t.dim() > 2:
        shape = [1] * (t.dim() - 1) + [w.numel()]
        return _w(torch.where(t > 0, t, t * w.reshape(shape)))
    return _w(TF.prelu(t, w))


def rrelu(x, lower=1. / 8., upper=1. / 3., training=True, name=None):
    return _w(TF.rrelu(_u(x), lower, upper, training))


def maxout(x, groups, axis=1, name=None):
    t = _u(x)
    axis = axis % t.dim()
    shp = list(t.shape)
    c = shp[axis]
    shp = shp[:axis] + [c // groups, groups] + shp[axis + 1:]
    return _w(t.reshape(shp).amax(axis + 1))


def glu(x, axis=-1, name=None):
    return _w(TF.glu(_u(x), axis))


@_amp_op('softmax')
def softmax(x, axis=-1, dtype=None, name=None):
    t = _u(x)
    if dtype is not None:
        t = t.to(_dt.to_torch_dtype(dtype))
    if ops.use_hip(t) and (axis == -1 or axis == t.dim() - 1):
        return _w(ops.softmax.softmax(t))
    return _w(torch.softmax(t, axis))


def softmax_(x, axis=-1, dtype=None, name=None):
    x._t = softmax(x, axis, dtype)._t
    return x


@_amp_op('log_softmax')
def log_softmax(x, axis=-1, dtype=None, name=None):
    t = _u(x)
    if dtype is not None:
        t = t.to(_dt.to_torch_dtype(dtype))
    return _w(torch.log_softmax(t, axis))


def gumbel_softmax(x, temperature=1.0, hard=False, axis=-1, name=None):
    return _w(TF.gumbel_softmax(_u(x), tau=temperature, hard=hard, dim=axis))


def swiglu(x, y=None, name=None):
    """paddle.incubate.nn.functional.swiglu: silu(x) * y (y=None → split x in half)."""
    t = _u(x)
    if y is None and ops.use_hip(t) and ops.act.swiglu_packed_ok(t):
        return _w(ops.act.swiglu_packed(t))  # one [rows, 2C] gradient, no chunk()/cat in autograd
    if y is None:
        a, b = t.chunk(2, dim=-1)
    else:
        a, b = t, _u(y)
    if ops.use_hip(a):
        return _w(ops.act.swiglu(a, b))
    return _w(TF.silu(a) * b)
