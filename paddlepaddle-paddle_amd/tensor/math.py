"""paddle math API (reference: python/paddle/tensor/math.py, python/paddle/tensor/ops.py).

Element-wise and reduction ops map onto the storage layer's kernels (ATen/HIP); the hot
fused ops used by the models live in ``ops/`` as hand-written HIP kernels.
"""
import builtins
import math as _pymath

import torch

from ._helpers import _w, _u, _t, _axis, _dims, _dtype, _scalar, Tensor
from ..core import dtype as _dt
from ..core.amp_dispatch import amp_op as _amp_op

# ----------------------------------------------------------------------------- unary
_UNARY = {
    'abs': torch.abs, 'acos': torch.acos, 'acosh': torch.acosh, 'asin': torch.asin, 'asinh': torch.asinh,
    'atan': torch.atan, 'atanh': torch.atanh, 'ceil': torch.ceil, 'cos': torch.cos, 'cosh': torch.cosh,
    'exp': torch.exp, 'expm1': torch.expm1, 'floor': torch.floor, 'log': torch.log, 'log2': torch.log2,
    'log10': torch.log10, 'log1p': torch.log1p, 'reciprocal': torch.reciprocal,
    'rsqrt': torch.rsqrt, 'sin': torch.sin, 'sinh': torch.sinh, 'sqrt': torch.sqrt, 'square': torch.square,
    'tan': torch.tan, 'tanh': torch.tanh, 'sigmoid': torch.sigmoid, 'trunc': torch.trunc, 'erf': torch.erf,
    'erfinv': torch.erfinv, 'sign': torch.sign, 'sgn': torch.sgn, 'neg': torch.neg, 'lgamma': torch.lgamma,
    'digamma': torch.digamma, 'frac': torch.frac, 'conj': torch.conj_physical, 'angle': torch.angle,
    'i0': torch.i0, 'i0e': torch.special.i0e, 'i1': torch.special.i1, 'i1e': torch.special.i1e,
    'sinc': torch.sinc, 'signbit': torch.signbit, 'deg2rad': torch.deg2rad, 'rad2deg': torch.rad2deg,
    'isfinite': torch.isfinite, 'isinf': torch.isinf, 'isnan': torch.isnan, 'isneginf': torch.isneginf,
    'isposinf': torch.isposinf, 'isreal': torch.isreal, 'bitwise_not': torch.bitwise_not,
    'logical_not': torch.logical_not, 'exp2': torch.exp2, 'gammaln': torch.lgamma,
}


def _make_unary(fn, name):
    def f(x, name=None):
        return _w(fn(x._t if isinstance(x, Tensor) else torch.as_tensor(x)))
    f.__name__ = name
    f.__doc__ = f"paddle.{name} (reference: python/paddle/tensor/math.py / ops.py)"
    return f


def _make_unary_(fn, name):
    inplace = getattr(torch.Tensor, name + '_', None)

    def f_(x, name=None):
        if inplace is not None:
            inplace(x._t)
        else:
            x._t.copy_(fn(x._t))
        return x
    f_.__name__ = name + '_'
    return f_


_UNARY_AMP = {'tan': 'tan', 'acos': 'acos', 'asin': 'asin', 'sinh': 'sinh', 'cosh': 'cosh', 'atanh': 'atanh',
              'erfinv': 'erfinv', 'exp': 'exp', 'expm1': 'expm1', 'log': 'log', 'log10': 'log10', 'log2': 'log2',
              'reciprocal': 'reciprocal', 'rsqrt': 'rsqrt', 'square': 'square'}  # reference FP16_BLACK_LIST names

for _n, _f in _UNARY.items():
    globals()[_n] = _make_unary(_f, _n)
    if _n in _UNARY_AMP:
        globals()[_n] = _amp_op(_UNARY_AMP[_n])(globals()[_n])
    if _n not in ('isfinite', 'isinf', 'isnan', 'isneginf', 'isposinf', 'isreal', 'signbit', 'angle', 'conj'):
        globals()[_n + '_'] = _make_unary_(_f, _n)


def round(x, decimals=0, name=None):  # noqa: A001
    return _w(torch.round(_u(x), decimals=decimals))


def round_(x, decimals=0, name=None):
    x._t.round_(decimals=decimals)
    return x


def logit(x, eps=None, name=None):
    return _w(torch.logit(_u(x), eps=eps))


def logit_(x, eps=None, name=None):
    x._t.logit_(eps=eps)
    return x


def polygamma(x, n, name=None):
    return _w(torch.polygamma(n, _u(x)))


def polygamma_(x, n, name=None):
    x._t.polygamma_(n)
    return x


def multigammaln(x, p, name=None):
    return _w(torch.mvlgamma(_u(x), p))


def multigammaln_(x, p, name=None):
    x._t.mvlgamma_(p)
    return x


def stanh(x, scale_a=0.67, scale_b=1.7159, name=None):
    return _w(scale_b * torch.tanh(scale_a * _u(x)))


def scale(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    s = _scalar(scale)
    t = _u(x)
    out = t * s + bias if bias_after_scale else (t + bias) * s
    if out.dtype != t.dtype and not isinstance(s, torch.Tensor):
        out = out.to(t.dtype)
    if act is not None:
        from ..nn import functional as F
        return getattr(F, act)(_w(out))
    return _w(out)


def scale_(x, scale=1.0, bias=0.0, bias_after_scale=True, act=None, name=None):
    s = _scalar(scale)
    if bias_after_scale:
        x._t.mul_(s).add_(bias)
    else:
        x._t.add_(bias).mul_(s)
    return x


@_amp_op('pow')
def pow(x, y, name=None):  # noqa: A001
    return _w(torch.pow(_t(x), _t(y, _u(x) if isinstance(x, Tensor) else None)))


def pow_(x, y, name=None):
    x._t.pow_(_t(y))
    return x


def float_power(x, y, name=None):
    return _w(torch.float_power(_t(x), _t(y)))


# ----------------------------------------------------------------------------- binary
def _binary(fn, name):
    def f(x, y, name=None):
        a = x._t if isinstance(x, Tensor) else x
        b = y._t if isinstance(y, Tensor) else y
        if not isinstance(a, torch.Tensor):
            a = torch.as_tensor(a, device=b.device if isinstance(b, torch.Tensor) else None)
        return _w(fn(a, _t(b, a)))
    f.__name__ = name
    return f


def _binary_(method, name):
    def f_(x, y, name=None):
        getattr(x._t, method)(_t(y, x._t))
        return x
    f_.__name__ = name + '_'
    return f_


_BINARY = {
    'add': (torch.add, 'add_'), 'subtract': (torch.sub, 'sub_'), 'multiply': (torch.mul, 'mul_'),
    'divide': (torch.true_divide, 'true_divide_'), 'floor_divide': (torch.floor_divide, 'floor_divide_'),
    'remainder': (torch.remainder, 'remainder_'), 'maximum': (torch.maximum, None), 'minimum': (torch.minimum, None),
    'fmax': (torch.fmax, None), 'fmin': (torch.fmin, None), 'atan2': (torch.atan2, 'atan2_'),
    'hypot': (torch.hypot, 'hypot_'), 'copysign': (torch.copysign, 'copysign_'), 'nextafter': (torch.nextafter, None),
    'heaviside': (torch.heaviside, None), 'gcd': (torch.gcd, 'gcd_'), 'lcm': (torch.lcm, 'lcm_'),
    'logaddexp': (torch.logaddexp, None), 'ldexp': (torch.ldexp, 'ldexp_'),
    'bitwise_and': (torch.bitwise_and, 'bitwise_and_'), 'bitwise_or': (torch.bitwise_or, 'bitwise_or_'),
    'bitwise_xor': (torch.bitwise_xor, 'bitwise_xor_'),
    'bitwise_left_shift': (torch.bitwise_left_shift, 'bitwise_left_shift_'),
    'bitwise_right_shift': (torch.bitwise_right_shift, 'bitwise_right_shift_'),
}
for _n, (_f, _m) in _BINARY.items():
    globals()[_n] = _binary(_f, _n)
    if _m is not None:
        globals()[_n + '_'] = _binary_(_m, _n)

mod = remainder  # noqa: F821
mod_ = remainder_  # noqa: F821
floor_mod = remainder  # noqa: F821
floor_mod_ = remainder_  # noqa: F821
elementwise_add = add  # noqa: F821


def lerp(x, y, weight, name=None):
    return _w(torch.lerp(_u(x), _u(y), _t(weight)))


def lerp_(x, y, weight, name=None):
    x._t.lerp_(_u(y), _t(weight))
    return x


def add_n(inputs, name=None):
    if isinstance(inputs, Tensor):
        return inputs
    out = inputs[0]._t
    for i in inputs[1:]:
        out = out + i._t
    return _w(out)


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):  # noqa: A002
    from ..ops import matmul as _hm
    return _w(_hm.addmm(_u(input), _u(x), _u(y), beta=beta, alpha=alpha))


def addmm_(input, x, y, beta=1.0, alpha=1.0, name=None):  # noqa: A002
    input._t.addmm_(_u(x), _u(y), beta=beta, alpha=alpha)
    return input


def baddbmm(input, x, y, beta=1.0, alpha=1.0, name=None):  # noqa: A002
    return _w(torch.baddbmm(_u(input), _u(x), _u(y), beta=beta, alpha=alpha))


def clip(x, min=None, max=None, name=None):  # noqa: A002
    return _w(torch.clamp(_u(x), _scalar(min), _scalar(max)))


def clip_(x, min=None, max=None, name=None):  # noqa: A002
    x._t.clamp_(_scalar(min), _scalar(max))
    return x


def nan_to_num(x, nan=0.0, posinf=None, neginf=None, name=None):
    return _w(torch.nan_to_num(_u(x), nan, posinf, neginf))


def nan_to_num_(x, nan=0.0, posinf=None, neginf=None, name=None):
    x._t.nan_to_num_(nan, posinf, neginf)
    return x


def increment(x, value=1.0, name=None):
    x._t.add_(value)
    return x


def frexp(x, name=None):
    m, e = torch.frexp(_u(x))
    return _w(m), _w(e.to(_u(x).dtype))


# ----------------------------------------------------------------------------- reductions
def _reduce(fn, x, axis, keepdim, dtype=None):
    t = _u(x)
    if dtype is not None:
        t = t.to(_dtype(dtype))
    a = _axis(axis)
    if a is None:
        r = fn(t)
        if keepdim:
            r = r.reshape([1] * t.dim())
        return _w(r)
    return _w(fn(t, dim=a, keepdim=keepdim))


@_amp_op('reduce_sum')
def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    t = _u(x)
    if dtype is None and (t.dtype == torch.bool or (not t.is_floating_point() and not t.is_complex() and t.dtype != torch.int64)):
        t = t.to(torch.int64)
    elif dtype is not None:
        t = t.to(_dtype(dtype))
    a = _axis(axis)
    if a is None:
        r = torch.sum(t)
        return _w(r.reshape([1] * t.dim()) if keepdim else r)
    return _w(torch.sum(t, dim=a, keepdim=keepdim))


def nansum(x, axis=None, dtype=None, keepdim=False, name=None):
    return _reduce(torch.nansum, x, axis, keepdim, dtype)


@_amp_op('mean')
def mean(x, axis=None, keepdim=False, name=None):
    return _reduce(torch.mean, x, axis, keepdim)


def nanmean(x, axis=None, keepdim=False, name=None):
    return _reduce(torch.nanmean, x, axis, keepdim)


@_amp_op('reduce_prod')
def prod(x, axis=None, keepdim=False, dtype=None, name=None):
    t = _u(x)
    if dtype is not None:
        t = t.to(_dtype(dtype))
    dims = _dims(axis, t.dim())
    r = t
    for d in sorted([d % builtins.max(t.dim(), 1) for d in dims], reverse=True):
        r = torch.prod(r, dim=d, keepdim=keepdim) if t.dim() else r
    if _axis(axis) is None and not keepdim:
        r = r.reshape([])
    return _w(r)


def _minmax(fn, x, axis, keepdim):
    t = _u(x)
    a = _axis(axis)
    if a is None:
        r = fn(t)
        return _w(r.reshape([1] * t.dim()) if keepdim else r)
    if isinstance(a, int):
        return _w(fn(t, dim=a, keepdim=keepdim)[0] if fn in (torch.max, torch.min) else fn(t, dim=a, keepdim=keepdim))
    return _w((torch.amax if fn is torch.max else torch.amin)(t, dim=a, keepdim=keepdim))


def max(x, axis=None, keepdim=False, name=None):  # noqa: A001
    return _minmax(torch.max, x, axis, keepdim)


def min(x, axis=None, keepdim=False, name=None):  # noqa: A001
    return _minmax(torch.min, x, axis, keepdim)


def amax(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    a = _axis(axis)
    return _w(torch.amax(t, dim=() if a is None else a, keepdim=keepdim))


def amin(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    a = _axis(axis)
    return _w(torch.amin(t, dim=() if a is None else a, keepdim=keepdim))


def all(x, axis=None, keepdim=False, name=None):  # noqa: A001
    t = _u(x)
    a = _axis(axis)
    if a is None:
        r = torch.all(t)
        return _w(r.reshape([1] * t.dim()) if keepdim else r)
    return _w(torch.all(t, dim=a, keepdim=keepdim))


def any(x, axis=None, keepdim=False, name=None):  # noqa: A001
    t = _u(x)
    a = _axis(axis)
    if a is None:
        r = torch.any(t)
        return _w(r.reshape([1] * t.dim()) if keepdim else r)
    return _w(torch.any(t, dim=a, keepdim=keepdim))


def logsumexp(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    return _w(torch.logsumexp(t, dim=_dims(axis, t.dim()), keepdim=keepdim))


def count_nonzero(x, axis=None, keepdim=False, name=None):
    t = _u(x)
    a = _axis(axis)
    r = torch.count_nonzero(t, dim=a)
    if keepdim:
        for d in sorted(_dims(axis, t.dim())):
            r = r.unsqueeze(d % t.dim())
    return _w(r)


@_amp_op('cumsum')
def cumsum(x, axis=None, dtype=None, name=None):
    t = _u(x)
    if axis is None:
        t = t.flatten()
        axis = 0
    return _w(torch.cumsum(t, dim=int(axis), dtype=_dtype(dtype)))


def cumsum_(x, axis=None, dtype=None, name=None):
    x._t.copy_(cumsum(x, axis, dtype)._t.reshape(x._t.shape))
    return x


@_amp_op('cumprod')
def cumprod(x, dim=None, dtype=None, name=None):
    t = _u(x)
    if dim is None:
        t = t.flatten()
        dim = 0
    return _w(torch.cumprod(t, dim=int(dim), dtype=_dtype(dtype)))


def cumprod_(x, dim=None, dtype=None, name=None):
    x._t.copy_(cumprod(x, dim, dtype)._t.reshape(x._t.shape))
    return x


def cummax(x, axis=None, dtype='int64', name=None):
    t = _u(x)
    if axis is None:
        t = t.flatten()
        axis = 0
    v, i = torch.cummax(t, dim=int(axis))
    return _w(v), _w(i.to(_dtype(dtype)))


def cummin(x, axis=None, dtype='int64', name=None):
    t = _u(x)
    if axis is None:
        t = t.flatten()
        axis = 0
    v, i = torch.cummin(t, dim=int(axis))
    return _w(v), _w(i.to(_dtype(dtype)))


def logcumsumexp(x, axis=None, dtype=None, name=None):
    t = _u(x)
    if dtype is not None:
        t = t.to(_dtype(dtype))
    if axis is None:
        t = t.flatten()
        axis = 0
    return _w(torch.logcumsumexp(t, dim=int(axis)))


def diff(x, n=1, axis=-1, prepend=None, append=None, name=None):
    return _w(torch.diff(_u(x), n=n, dim=axis, prepend=_u(prepend), append=_u(append)))


def trace(x, offset=0, axis1=0, axis2=1, name=None):
    return _w(torch.diagonal(_u(x), offset=offset, dim1=axis1, dim2=axis2).sum(-1))


def kron(x, y, name=None):
    return _w(torch.kron(_u(x), _u(y)))


def inner(x, y, name=None):
    return _w(torch.inner(_u(x), _u(y)))


def outer(x, y, name=None):
    return _w(torch.outer(_u(x).flatten(), _u(y).flatten()))


def cross(x, y, axis=9, name=None):
    t = _u(x)
    if axis == 9:
        axis = next(i for i, s in enumerate(t.shape) if s == 3)
    return _w(torch.linalg.cross(t, _u(y), dim=axis))


@_amp_op('renorm')
def renorm(x, p, axis, max_norm, name=None):
    return _w(torch.renorm(_u(x), p, axis, max_norm))


def renorm_(x, p, axis, max_norm, name=None):
    x._t.renorm_(p, axis, max_norm)
    return x


def gammainc(x, y, name=None):
    return _w(torch.special.gammainc(_u(x), _u(y)))


def gammaincc(x, y, name=None):
    return _w(torch.special.gammaincc(_u(x), _u(y)))


def gammainc_(x, y, name=None):
    x._t.copy_(torch.special.gammainc(x._t, _u(y)))
    return x


def gammaincc_(x, y, name=None):
    x._t.copy_(torch.special.gammaincc(x._t, _u(y)))
    return x


def trapezoid(y, x=None, dx=None, axis=-1, name=None):
    if x is not None:
        return _w(torch.trapezoid(_u(y), _u(x), dim=axis))
    return _w(torch.trapezoid(_u(y), dx=1.0 if dx is None else dx, dim=axis))


def cumulative_trapezoid(y, x=None, dx=None, axis=-1, name=None):
    if x is not None:
        return _w(torch.cumulative_trapezoid(_u(y), _u(x), dim=axis))
    return _w(torch.cumulative_trapezoid(_u(y), dx=1.0 if dx is None else dx, dim=axis))


def vander(x, n=None, increasing=False, name=None):
    return _w(torch.linalg.vander(_u(x), N=n) if increasing else torch.linalg.vander(_u(x), N=n).flip(-1))


def isclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return _w(torch.isclose(_u(x), _u(y), rtol=rtol, atol=atol, equal_nan=equal_nan))


def allclose(x, y, rtol=1e-05, atol=1e-08, equal_nan=False, name=None):
    return _w(torch.tensor(torch.allclose(_u(x), _t(y, _u(x)), rtol=rtol, atol=atol, equal_nan=equal_nan)))


def broadcast_shape(x_shape, y_shape):
    return list(torch.broadcast_shapes(tuple(x_shape), tuple(y_shape)))


def inverse(x, name=None):
    return _w(torch.linalg.inv(_u(x)))


def log_normal_(x, mean=1.0, std=2.0, name=None):
    x._t.log_normal_(mean, std)
    return x


def combinations(x, r=2, with_replacement=False, name=None):
    return _w(torch.combinations(_u(x), r=r, with_replacement=with_replacement))


def take(x, index, mode='raise', name=None):
    t = _u(x).flatten()
    i = _u(index)
    n = t.numel()
    if mode == 'wrap':
        i = torch.remainder(i, n)
    elif mode == 'clip':
        i = torch.clamp(i, 0, n - 1)
    else:
        i = torch.where(i < 0, i + n, i)
    return _w(t[i])


def reduce_as(x, target, name=None):
    t, tg = _u(x), _u(target)
    nd = t.dim() - tg.dim()
    r = t.sum(dim=tuple(range(nd))) if nd > 0 else t
    dims = tuple(i for i, (a, b) in enumerate(zip(r.shape, tg.shape)) if a != b and b == 1)
    if dims:
        r = r.sum(dim=dims, keepdim=True)
    return _w(r)


def signbit_(x):
    return _w(torch.signbit(_u(x)))


def sqrt_int(n):
    return _pymath.isqrt(n)


def neg_(x, name=None):
    x._t.neg_()
    return x


def tanh_(x, name=None):
    x._t.tanh_()
    return x


def is_empty(x, name=None):
    return _w(torch.tensor(_u(x).numel() == 0))


def numel(x, name=None):
    return _w(torch.tensor(_u(x).numel(), dtype=torch.int64))


def is_floating_point(x):
    return _u(x).is_floating_point()


def is_complex(x):
    return _u(x).is_complex()


def is_integer(x):
    return _dt.is_integer_dtype(_u(x).dtype)


def rank(input):  # noqa: A002
    return _w(torch.tensor(_u(input).dim(), dtype=torch.int32))


@_amp_op('dist')
def dist(x, y, p=2, name=None):
    return _w(torch.dist(_u(x), _u(y), p=p))


def hsigmoid_(x):
    return _w(torch.nn.functional.hardsigmoid(_u(x)))


def real(x, name=None):
    """Real part (reference python/paddle/tensor/attribute.py real); a copy, like the reference."""
    t = _u(x)
    return _w(torch.real(t).clone() if t.is_complex() else t.clone())


def imag(x, name=None):
    """Imaginary part (reference python/paddle/tensor/attribute.py imag)."""
    t = _u(x)
    return _w(torch.imag(t).clone() if t.is_complex() else torch.zeros_like(t))
