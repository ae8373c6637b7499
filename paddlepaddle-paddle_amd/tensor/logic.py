"""paddle logic / search / stat / random APIs
(reference: python/paddle/tensor/{logic,search,stat,random}.py)."""
import builtins

import torch

from ._helpers import _w, _u, _t, _axis, _dims, _shape, _dtype, _scalar, Tensor
from ..core import dtype as _dt
from ..core.place import current_device


def _cmp(fn, name):
    def f(x, y, name=None):
        a = _u(x)
        return _w(fn(a, _t(y, a)))
    f.__name__ = name
    return f


def _cmp_(fn, name):
    def f_(x, y, name=None):
        x._t = fn(x._t, _t(y, x._t))
        return x
    f_.__name__ = name + '_'
    return f_


for _n, _f in {'equal': torch.eq, 'not_equal': torch.ne, 'less_than': torch.lt, 'less_equal': torch.le,
               'greater_than': torch.gt, 'greater_equal': torch.ge, 'logical_and': torch.logical_and,
               'logical_or': torch.logical_or, 'logical_xor': torch.logical_xor}.items():
    globals()[_n] = _cmp(_f, _n)
    globals()[_n + '_'] = _cmp_(_f, _n)

less = globals()['less_than']
greater = globals()['greater_than']


def logical_not_(x, name=None):
    x._t = torch.logical_not(x._t)
    return x


def equal_all(x, y, name=None):
    a, b = _u(x), _u(y)
    return _w(torch.tensor(a.shape == b.shape and bool(torch.equal(a, b)), device=a.device))


def is_tensor(x):
    return isinstance(x, Tensor)


def isin(x, test_x, assume_unique=False, invert=False, name=None):
    return _w(torch.isin(_u(x), _u(test_x), assume_unique=assume_unique, invert=invert))


# ----------------------------------------------------------------------------- search
def argmax(x, axis=None, keepdim=False, dtype='int64', name=None):
    t = _u(x)
    if axis is None:
        r = torch.argmax(t.flatten())
        return _w((r.reshape([1] * t.dim()) if keepdim else r).to(_dtype(dtype)))
    return _w(torch.argmax(t, dim=int(axis), keepdim=keepdim).to(_dtype(dtype)))


def argmin(x, axis=None, keepdim=False, dtype='int64', name=None):
    t = _u(x)
    if axis is None:
        r = torch.argmin(t.flatten())
        return _w((r.reshape([1] * t.dim()) if keepdim else r).to(_dtype(dtype)))
    return _w(torch.argmin(t, dim=int(axis), keepdim=keepdim).to(_dtype(dtype)))


def argsort(x, axis=-1, descending=False, stable=False, name=None):
    return _w(torch.argsort(_u(x), dim=axis, descending=descending, stable=stable))


def sort(x, axis=-1, descending=False, stable=False, name=None):
    return _w(torch.sort(_u(x), dim=axis, descending=descending, stable=stable)[0])


def topk(x, k, axis=None, largest=True, sorted=True, name=None):  # noqa: A002
    k = int(_scalar(k))
    v, i = torch.topk(_u(x), k, dim=-1 if axis is None else axis, largest=largest, sorted=sorted)
    return _w(v), _w(i)


def where(condition, x=None, y=None, name=None):
    c = _u(condition)
    if x is None and y is None:
        return nonzero(condition, as_tuple=True)
    a = _t(x, c)
    b = _t(y, c)
    if not isinstance(a, torch.Tensor):
        a = torch.tensor(a, device=c.device, dtype=b.dtype if isinstance(b, torch.Tensor) else None)
    if not isinstance(b, torch.Tensor):
        b = torch.tensor(b, device=c.device, dtype=a.dtype)
    return _w(torch.where(c, a, b))


def where_(condition, x=None, y=None, name=None):
    x._t.copy_(where(condition, x, y)._t)
    return x


def nonzero(x, as_tuple=False):
    t = _u(x)
    if as_tuple:
        return tuple(_w(i.unsqueeze(-1)) for i in torch.nonzero(t, as_tuple=True))
    return _w(torch.nonzero(t))


def searchsorted(sorted_sequence, values, out_int32=False, right=False, name=None):
    return _w(torch.searchsorted(_u(sorted_sequence), _u(values), out_int32=out_int32, right=right))


def bucketize(x, sorted_sequence, out_int32=False, right=False, name=None):
    return _w(torch.bucketize(_u(x), _u(sorted_sequence), out_int32=out_int32, right=right))


def kthvalue(x, k, axis=None, keepdim=False, name=None):
    v, i = torch.kthvalue(_u(x), k, dim=-1 if axis is None else axis, keepdim=keepdim)
    return _w(v), _w(i)


def mode(x, axis=-1, keepdim=False, name=None):
    v, i = torch.mode(_u(x), dim=axis, keepdim=keepdim)
    return _w(v), _w(i)


def top_p_sampling(x, ps, threshold=None, topp_seed=None, seed=-1, k=0, mode='truncated', return_top=False, name=None):
    probs = _u(x)
    sp, si = torch.sort(probs, dim=-1, descending=True)
    cum = sp.cumsum(-1)
    p = _u(ps).reshape(-1, 1)
    mask = cum - sp > p
    sp = sp.masked_fill(mask, 0)
    choice = torch.multinomial(sp / sp.sum(-1, keepdim=True), 1)
    ids = si.gather(-1, choice)
    return _w(probs.gather(-1, ids)), _w(ids)


# ----------------------------------------------------------------------------- stat
def var(x, axis=None, unbiased=True, keepdim=False, name=None):
    t = _u(x)
    return _w(torch.var(t, dim=_axis(axis), unbiased=unbiased, keepdim=keepdim))


def std(x, axis=None, unbiased=True, keepdim=False, name=None):
    t = _u(x)
    return _w(torch.std(t, dim=_axis(axis), unbiased=unbiased, keepdim=keepdim))


def median(x, axis=None, keepdim=False, mode='avg', name=None):
    t = _u(x)
    if mode == 'min':
        if axis is None:
            return _w(torch.median(t.flatten()))
        v, i = torch.median(t, dim=axis, keepdim=keepdim)
        return _w(v), _w(i)
    if axis is None:
        r = torch.quantile(t.flatten().to(torch.float64 if t.dtype == torch.float64 else torch.float32), 0.5)
        return _w((r.reshape([1] * t.dim()) if keepdim else r).to(t.dtype if t.is_floating_point() else torch.float32))
    r = torch.quantile(t.float() if not t.is_floating_point() else t, 0.5, dim=axis, keepdim=keepdim)
    return _w(r)


def nanmedian(x, axis=None, keepdim=False, mode='avg', name=None):
    t = _u(x)
    if axis is None:
        return _w(torch.nanquantile(t.flatten(), 0.5))
    return _w(torch.nanquantile(t, 0.5, dim=axis, keepdim=keepdim))


def quantile(x, q, axis=None, keepdim=False, interpolation='linear', name=None):
    t = _u(x)
    qq = torch.tensor(q, dtype=t.dtype, device=t.device) if isinstance(q, (list, tuple)) else q
    a = _axis(axis)
    if isinstance(a, tuple):
        t = t.movedim(a, tuple(range(-len(a), 0))).flatten(-len(a))
        a = -1
    return _w(torch.quantile(t, qq, dim=a, keepdim=keepdim, interpolation=interpolation))


def nanquantile(x, q, axis=None, keepdim=False, interpolation='linear', name=None):
    t = _u(x)
    qq = torch.tensor(q, dtype=t.dtype, device=t.device) if isinstance(q, (list, tuple)) else q
    return _w(torch.nanquantile(t, qq, dim=_axis(axis), keepdim=keepdim, interpolation=interpolation))


# ----------------------------------------------------------------------------- random
def _fdt(dtype):
    return _dtype(dtype) if dtype is not None else _dt.default_float()


def rand(shape, dtype=None, name=None):
    return _w(torch.rand(_shape(shape), dtype=_fdt(dtype), device=current_device()))


def randn(shape, dtype=None, name=None):
    return _w(torch.randn(_shape(shape), dtype=_fdt(dtype), device=current_device()))


standard_normal = randn


def randint(low=0, high=None, shape=[1], dtype=None, name=None):  # noqa: B006
    if high is None:
        low, high = 0, low
    return _w(torch.randint(low, high, _shape(shape), dtype=_dtype(dtype) or torch.int64, device=current_device()))


def randint_like(x, low=0, high=None, dtype=None, name=None):
    if high is None:
        low, high = 0, low
    t = _u(x)
    return _w(torch.randint(low, high, t.shape, dtype=_dtype(dtype) or t.dtype, device=t.device))


def randperm(n, dtype='int64', name=None):
    return _w(torch.randperm(n, dtype=_dtype(dtype), device=current_device()))


def uniform(shape, dtype=None, min=-1.0, max=1.0, seed=0, name=None):  # noqa: A002
    t = torch.empty(_shape(shape), dtype=_fdt(dtype), device=current_device())
    if seed:
        g = torch.Generator(device=t.device).manual_seed(seed)
        return _w(t.uniform_(min, max, generator=g))
    return _w(t.uniform_(min, max))


def uniform_(x, min=-1.0, max=1.0, seed=0, name=None):  # noqa: A002
    with torch.no_grad():
        x._t.uniform_(min, max)
    return x


def normal(mean=0.0, std=1.0, shape=None, name=None):
    if isinstance(mean, Tensor) or isinstance(std, Tensor):
        m, s = _u(mean), _u(std)
        return _w(torch.normal(m if isinstance(m, torch.Tensor) else torch.full_like(s, m),
                               s if isinstance(s, torch.Tensor) else torch.full_like(m, s)))
    return _w(torch.normal(mean, std, _shape(shape), device=current_device(), dtype=_dt.default_float()))


def normal_(x, mean=0.0, std=1.0, name=None):
    with torch.no_grad():
        x._t.normal_(mean, std)
    return x


def gaussian(shape, mean=0.0, std=1.0, seed=0, dtype=None, name=None):
    return _w(torch.normal(mean, std, _shape(shape), device=current_device(), dtype=_fdt(dtype)))


def log_normal(mean=1.0, std=2.0, shape=None, name=None):
    return _w(torch.empty(_shape(shape), device=current_device()).log_normal_(mean, std))


def bernoulli(x, p=None, name=None):
    t = _u(x)
    return _w(torch.bernoulli(t if p is None else torch.full_like(t, p)))


def bernoulli_(x, p=0.5, name=None):
    with torch.no_grad():
        x._t.bernoulli_(_t(p))
    return x


def binomial(count, prob, name=None):
    return _w(torch.binomial(_u(count).float(), _u(prob).float()).to(torch.int64))


def poisson(x, name=None):
    return _w(torch.poisson(_u(x)))


def standard_gamma(x, name=None):
    return _w(torch._standard_gamma(_u(x)))


def multinomial(x, num_samples=1, replacement=False, name=None):
    return _w(torch.multinomial(_u(x), num_samples, replacement))


def exponential_(x, lam=1.0, name=None):
    with torch.no_grad():
        x._t.exponential_(lam)
    return x


def cauchy_(x, loc=0, scale=1, name=None):
    with torch.no_grad():
        x._t.cauchy_(loc, scale)
    return x


def geometric_(x, probs, name=None):
    with torch.no_grad():
        x._t.geometric_(_scalar(probs))
    return x


def rrelu_noise(x, lower, upper):
    return torch.empty_like(x).uniform_(lower, upper)


def dims_of(axis, nd):
    return _dims(axis, nd)


_ = builtins
