"""paddle.autograd (reference: python/paddle/autograd/{__init__,py_layer,backward_mode,autograd}.py).

Backward runs on torch's autograd engine over the storage tensors; this module adds the
paddle surface: ``paddle.grad``, ``backward``, ``PyLayer`` (custom forward/backward),
``no_grad``/``enable_grad``/``set_grad_enabled`` and ``jacobian``/``hessian``.
"""
import functools

import torch

from ..core.tensor import Tensor, _wrap, _unwrap


class no_grad:
    """Context manager *and* decorator (paddle.no_grad / paddle.base.dygraph.no_grad)."""

    def __init__(self, func=None):
        self._func = func
        if func is not None:
            functools.update_wrapper(self, func)

    def __call__(self, *args, **kwargs):
        if self._func is not None:
            with torch.no_grad():
                return self._func(*args, **kwargs)
        func = args[0]

        @functools.wraps(func)
        def wrapper(*a, **k):
            with torch.no_grad():
                return func(*a, **k)
        return wrapper

    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(False)

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)


class enable_grad(no_grad):
    def __call__(self, *args, **kwargs):
        if self._func is not None:
            with torch.enable_grad():
                return self._func(*args, **kwargs)
        func = args[0]

        @functools.wraps(func)
        def wrapper(*a, **k):
            with torch.enable_grad():
                return func(*a, **k)
        return wrapper

    def __enter__(self):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(True)


class set_grad_enabled:
    def __init__(self, mode):
        self._prev = torch.is_grad_enabled()
        torch.set_grad_enabled(mode)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        torch.set_grad_enabled(self._prev)


def is_grad_enabled():
    return torch.is_grad_enabled()


def _tl(xs):
    if xs is None:
        return None
    if isinstance(xs, Tensor):
        return [xs._t]
    return [_unwrap(x) for x in xs]


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False, only_inputs=True,
         allow_unused=False, no_grad_vars=None):
    """paddle.grad (reference: python/paddle/base/dygraph/base.py:grad)."""
    single = isinstance(inputs, Tensor)
    outs = _tl(outputs)
    ins = _tl(inputs)
    gos = _tl(grad_outputs)
    if gos is not None:
        gos = [torch.ones_like(o) if g is None else g for o, g in zip(outs, gos)]
    else:
        gos = [torch.ones_like(o) for o in outs]
    if retain_graph is None:
        retain_graph = create_graph
    gs = torch.autograd.grad(outs, ins, gos, retain_graph=retain_graph, create_graph=create_graph,
                             allow_unused=allow_unused)
    res = [None if g is None else _wrap(g) for g in gs]
    return res if not single else res


def backward(tensors, grad_tensors=None, retain_graph=False):
    ts = _tl(tensors)
    gs = _tl(grad_tensors)
    torch.autograd.backward(ts, gs, retain_graph=retain_graph)


# ----------------------------------------------------------------------------- PyLayer
class PyLayerContext:
    """ctx object handed to PyLayer.forward/backward."""

    def __init__(self, tctx):
        self._tctx = tctx
        self.container = None
        self.not_inplace_tensors = ()
        self._materialize = True

    def save_for_backward(self, *tensors):
        self._tctx.save_for_backward(*[t._t if isinstance(t, Tensor) else None for t in tensors])
        self._saved = [None if isinstance(t, Tensor) else t for t in tensors]
        self._saved_kinds = [isinstance(t, Tensor) for t in tensors]

    def saved_tensor(self):
        return tuple(_wrap(t) if k else o
                     for t, k, o in zip(self._tctx.saved_tensors, self._saved_kinds, self._saved))

    def mark_not_inplace(self, *args):
        self.not_inplace_tensors = args

    def mark_non_differentiable(self, *args):
        self._tctx.mark_non_differentiable(*[_unwrap(a) for a in args])

    def set_materialize_grads(self, value):
        self._tctx.set_materialize_grads(value)


_setup_stack = []


def _make_fn(cls):
    class _Fn(torch.autograd.Function):
        @staticmethod
        def forward(tctx, *args):
            kinds, kwargs = _setup_stack.pop()
            tctx.kinds = kinds
            ctx = PyLayerContext(tctx)
            tctx.pctx = ctx
            wargs = [_wrap(a) if k else a for a, k in zip(args, kinds)]
            with torch.no_grad():
                out = cls.forward(ctx, *wargs, **kwargs)
            if isinstance(out, (tuple, list)):
                return tuple(_unwrap(o) for o in out)
            return _unwrap(out)

        @staticmethod
        def backward(tctx, *gouts):
            gs = cls.backward(tctx.pctx, *[None if g is None else _wrap(g) for g in gouts])
            if not isinstance(gs, (tuple, list)):
                gs = (gs,)
            res = []
            gi = iter(gs)
            for k in tctx.kinds:
                if k:
                    g = next(gi, None)
                    res.append(None if g is None else _unwrap(g))
                else:
                    res.append(None)
            return tuple(res)
    _Fn.__name__ = cls.__name__ + 'Backward'
    return _Fn


class PyLayerMeta(type):
    def __init__(cls, name, bases, attrs):
        super().__init__(name, bases, attrs)
        cls._fn = None


class PyLayer(metaclass=PyLayerMeta):
    """paddle.autograd.PyLayer: user-defined forward/backward (reference: autograd/py_layer.py)."""

    @staticmethod
    def forward(ctx, *args, **kwargs):
        raise NotImplementedError

    @staticmethod
    def backward(ctx, *args):
        raise NotImplementedError

    @classmethod
    def apply(cls, *args, **kwargs):
        if cls.__dict__.get('_fn') is None:
            cls._fn = _make_fn(cls)
        _setup_stack.append(([isinstance(a, Tensor) for a in args], kwargs))
        out = cls._fn.apply(*[_unwrap(a) for a in args])
        if isinstance(out, tuple):
            return tuple(_wrap(o) if isinstance(o, torch.Tensor) else o for o in out)
        return _wrap(out) if isinstance(out, torch.Tensor) else out


LegacyPyLayer = PyLayer
EagerPyLayer = PyLayer


def saved_tensors_hooks(pack_hook, unpack_hook):
    return torch.autograd.graph.saved_tensors_hooks(lambda t: pack_hook(_wrap(t)),
                                                    lambda p: _unwrap(unpack_hook(p)))


from .functional import jacobian, hessian, vjp, jvp, Jacobian, Hessian  # noqa: E402,F401
