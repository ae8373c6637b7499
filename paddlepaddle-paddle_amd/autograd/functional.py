"""paddle.autograd.{jacobian,hessian,vjp,jvp} (reference: python/paddle/autograd/autograd.py)."""
import torch

from ..core.tensor import Tensor, _wrap, _unwrap


def _call(func, xs):
    single = isinstance(xs, Tensor)
    tx = [xs._t] if single else [x._t for x in xs]

    def f(*args):
        r = func(*([_wrap(a) for a in args] if not single else [_wrap(args[0])]))
        return tuple(_unwrap(o) for o in r) if isinstance(r, (tuple, list)) else _unwrap(r)
    return f, tx, single


def vjp(func, xs, v=None):
    f, tx, single = _call(func, xs)
    out, g = torch.autograd.functional.vjp(f, tuple(tx), None if v is None else (
        _unwrap(v) if isinstance(v, Tensor) else tuple(_unwrap(e) for e in v)), create_graph=True)
    wrap = (lambda o: tuple(_wrap(e) for e in o) if isinstance(o, tuple) else _wrap(o))
    g = g[0] if single else g
    return wrap(out), wrap(g)


def jvp(func, xs, v=None):
    f, tx, single = _call(func, xs)
    out, g = torch.autograd.functional.jvp(f, tuple(tx), None if v is None else (
        (_unwrap(v),) if isinstance(v, Tensor) else tuple(_unwrap(e) for e in v)), create_graph=True)
    wrap = (lambda o: tuple(_wrap(e) for e in o) if isinstance(o, tuple) else _wrap(o))
    return wrap(out), wrap(g)


class Jacobian:
    """Lazily-evaluated Jacobian matrix (paddle.autograd.jacobian returns this)."""

    def __init__(self, ys_fn_or_t, xs, is_batched=False):
        self._value = ys_fn_or_t

    @property
    def shape(self):
        return list(self._value.shape)

    def __getitem__(self, idx):
        return _wrap(self._value[tuple(_unwrap(i) if isinstance(i, Tensor) else i for i in idx)
                                 if isinstance(idx, tuple) else idx])

    def numpy(self):
        return self._value.detach().cpu().numpy()


Hessian = Jacobian


def _jac_t(y, x, batch_axis=None):
    """d y / d x for torch tensors via repeated grad; flattened to 2-D (or 3-D batched)."""
    yf = y.reshape(-1) if batch_axis is None else y.reshape(y.shape[0], -1)
    rows = []
    n = yf.shape[-1]
    for i in range(n):
        gy = torch.zeros_like(yf)
        if batch_axis is None:
            gy[i] = 1
        else:
            gy[:, i] = 1
        g, = torch.autograd.grad(yf, x, gy.reshape(yf.shape), retain_graph=True, create_graph=True, allow_unused=True)
        g = torch.zeros_like(x) if g is None else g
        rows.append(g.reshape(-1) if batch_axis is None else g.reshape(g.shape[0], -1))
    return torch.stack(rows, dim=0 if batch_axis is None else 1)


def jacobian(ys, xs, batch_axis=None):
    ys_l = [ys] if isinstance(ys, Tensor) else list(ys)
    xs_l = [xs] if isinstance(xs, Tensor) else list(xs)
    res = [[Jacobian(_jac_t(y._t, x._t, batch_axis), x) for x in xs_l] for y in ys_l]
    if isinstance(ys, Tensor) and isinstance(xs, Tensor):
        return res[0][0]
    if isinstance(ys, Tensor):
        return tuple(res[0])
    if isinstance(xs, Tensor):
        return tuple(r[0] for r in res)
    return tuple(tuple(r) for r in res)


def hessian(ys, xs, batch_axis=None):
    xs_l = [xs] if isinstance(xs, Tensor) else list(xs)
    y = ys._t
    res = []
    for xi in xs_l:
        row = []
        g, = torch.autograd.grad(y.sum() if batch_axis is not None else y, xi._t, create_graph=True)
        for xj in xs_l:
            row.append(Jacobian(_jac_t(g, xj._t, batch_axis), xj))
        res.append(tuple(row))
    if isinstance(xs, Tensor):
        return res[0][0]
    return tuple(res)
