"""paddle.incubate.autograd (reference: python/paddle/incubate/autograd/{functional,primapi,utils}.py):
function-form Jacobian / Hessian matrices, vjp / jvp, forward-mode ``forward_grad``, reverse-mode
``grad`` and the primitive-operator switch.

``enable_prim()`` turns on composite-op decomposition for static programs: ``Executor.run``
rewrites a program through ``paddle.decomposition.decompose`` before its first run (the
reference lowers to primitive ops for its prim autodiff / compiler).
"""
import torch

from ..autograd.functional import vjp, jvp  # noqa: F401
from ..core.tensor import Tensor, _wrap, _unwrap

__all__ = ['vjp', 'jvp', 'Jacobian', 'Hessian', 'enable_prim', 'disable_prim', 'forward_grad', 'grad']

_PRIM = {'enabled': False}


def enable_prim():
    _PRIM['enabled'] = True
    from ..decomposition import decomp
    decomp._prim_config['prim_enabled'] = True


def disable_prim():
    _PRIM['enabled'] = False
    from ..decomposition import decomp
    decomp._prim_config['prim_enabled'] = False


def prim_enabled():
    return _PRIM['enabled']


def _flat_fn(func, xs, single):
    shapes = [x.shape for x in xs]
    sizes = [int(torch.tensor(s).prod()) if len(s) else 1 for s in shapes]

    def f(flat):
        parts, o = [], 0
        for s, n in zip(shapes, sizes):
            parts.append(flat[o:o + n].reshape(s))
            o += n
        args = [_wrap(p) for p in parts]
        r = func(args[0]) if single else func(*args)
        rs = r if isinstance(r, (tuple, list)) else [r]
        return torch.cat([_unwrap(t).reshape(-1) for t in rs])
    return f


class Jacobian:
    """J[i, j] = d out_i / d in_j of ``func`` at ``xs`` (inputs and outputs flattened and
    concatenated); ``is_batched``: the leading dim of every input/output is a batch → [B, M, N]."""

    def __init__(self, func, xs, is_batched=False):
        single = isinstance(xs, Tensor)
        xl = [xs] if single else list(xs)
        ts = [_unwrap(x).detach() for x in xl]
        if not is_batched:
            flat = torch.cat([t.reshape(-1) for t in ts])
            self._value = torch.autograd.functional.jacobian(_flat_fn(func, ts, single), flat, create_graph=True)
        else:
            B = ts[0].shape[0]
            rows = []
            for b in range(B):  # per-sample Jacobians (samples are independent by contract)
                tb = [t[b] for t in ts]
                flat = torch.cat([t.reshape(-1) for t in tb])

                def fb(fl, tb=tb, b=b):
                    parts, o = [], 0
                    for t in tb:
                        n = t.numel()
                        parts.append(fl[o:o + n].reshape(t.shape))
                        o += n
                    full = [torch.cat([ts[i][:b], parts[i][None], ts[i][b + 1:]]) for i in range(len(ts))]
                    r = func(_wrap(full[0])) if single else func(*[_wrap(p) for p in full])
                    rs = r if isinstance(r, (tuple, list)) else [r]
                    return torch.cat([_unwrap(t)[b].reshape(-1) for t in rs])
                rows.append(torch.autograd.functional.jacobian(fb, flat, create_graph=True))
            self._value = torch.stack(rows)

    @property
    def shape(self):
        return list(self._value.shape)

    def __getitem__(self, idx):
        return _wrap(self._value[idx])

    def numpy(self):
        return self._value.detach().cpu().numpy()


class Hessian(Jacobian):
    """H = d^2 func / d xs^2 of a scalar-valued ``func`` (flattened, concatenated inputs)."""

    def __init__(self, func, xs, is_batched=False):
        single = isinstance(xs, Tensor)
        xl = [xs] if single else list(xs)
        ts = [_unwrap(x).detach() for x in xl]
        if is_batched:
            super().__init__(lambda *a: _grad_of(func, a, single), xs, True)
            return
        flat = torch.cat([t.reshape(-1) for t in ts])
        self._value = torch.autograd.functional.hessian(_flat_fn(func, ts, single), flat, create_graph=True)


def _grad_of(func, args, single):
    ts = [_unwrap(a) for a in args]
    r = func(args[0]) if single else func(*args)
    g = torch.autograd.grad(_unwrap(r).sum(), ts, create_graph=True)
    return [_wrap(x) for x in g] if len(g) > 1 else _wrap(g[0])


def grad(outputs, inputs, grad_outputs=None):
    """Reverse-mode gradients of ``outputs`` w.r.t. ``inputs`` (create_graph, so it composes)."""
    from ..autograd import grad as _g
    single = isinstance(inputs, Tensor)
    r = _g(outputs, inputs, grad_outputs, create_graph=True, allow_unused=True)
    return r[0] if single and isinstance(r, (list, tuple)) else r


def forward_grad(outputs, inputs, grad_inputs=None):
    """Forward-mode derivative (jvp) of already-computed ``outputs`` along ``grad_inputs`` (ones by
    default): the transpose of the reverse-mode vjp, taken by differentiating the vjp w.r.t. its
    cotangent."""
    outs = [outputs] if isinstance(outputs, Tensor) else list(outputs)
    ins = [inputs] if isinstance(inputs, Tensor) else list(inputs)
    if grad_inputs is None:
        vs = [torch.ones_like(_unwrap(x)) for x in ins]
    else:
        vs = [_unwrap(v) for v in ([grad_inputs] if isinstance(grad_inputs, Tensor) else grad_inputs)]
    ys = [_unwrap(o) for o in outs]
    us = [torch.zeros_like(y, requires_grad=True) for y in ys]
    gx = torch.autograd.grad(ys, [_unwrap(x) for x in ins], us, create_graph=True, allow_unused=True)
    pairs = [(g, v) for g, v in zip(gx, vs) if g is not None]
    jv = torch.autograd.grad([g for g, _ in pairs], us, [v for _, v in pairs], create_graph=True, allow_unused=True)
    res = [_wrap(j if j is not None else torch.zeros_like(y)) for j, y in zip(jv, ys)]
    return res[0] if isinstance(outputs, Tensor) else res
