"""The eager ``paddle.Tensor``.

Reference: paddle/fluid/eager (core.eager.Tensor) + python/paddle/base/dygraph/tensor_patch_methods.py.

Design: a ``Tensor`` is a thin handle (``__slots__``) over a torch storage tensor ``_t``
living on the HIP device (or CPU).  Autograd is torch's engine: ``stop_gradient`` is the
inverse of ``_t.requires_grad``; the graph is recorded by the torch ops (and by our HIP
kernels' ``torch.autograd.Function`` wrappers) that produce ``_t``.  The handle adds the
paddle surface (list shapes, ``place``, ``stop_gradient``, ``numpy()``, ``name``,
``persistable`` …) without touching the storage, so every op costs one attribute load
to unwrap and one object allocation to wrap.
"""
import itertools

import numpy as np
import weakref

import torch

from . import dtype as _dt
from .place import current_device, place_of, to_device

_name_counter = itertools.count()


class Tensor:
    __slots__ = ('_t', '_name', 'persistable', '__weakref__', '__dict__')

    # ------------------------------------------------------------------ construction
    def __init__(self, value=None, dtype=None, place=None, persistable=False, zero_copy=False, name=None,
                 stop_gradient=True):
        if value is None:
            t = torch.empty(0)
        elif isinstance(value, Tensor):
            t = value._t
        elif isinstance(value, torch.Tensor):
            t = value
        else:
            t = _as_torch(value, dtype=dtype, device=to_device(place))
        if dtype is not None and t.dtype != _dt.to_torch_dtype(dtype):
            t = t.to(_dt.to_torch_dtype(dtype))
        if place is not None:
            t = t.to(to_device(place))
        if not stop_gradient and t.is_floating_point():
            t = t.detach().requires_grad_(True)
        self._t = t
        self._name = name
        self.persistable = persistable

    # ------------------------------------------------------------------ paddle attributes
    @property
    def name(self):
        if self._name is None:
            self._name = f"generated_tensor_{next(_name_counter)}"
        return self._name

    @name.setter
    def name(self, v):
        self._name = v

    @property
    def shape(self):
        t = self._t
        if t.is_meta:  # static-graph Variable: dynamic dims read as -1
            from ..static.program import static_shape
            return static_shape(t)
        return list(t.shape)

    @property
    def ndim(self):
        return self._t.dim()

    def dim(self):
        return self._t.dim()

    ndimension = dim

    @property
    def size(self):
        return self._t.numel()

    def numel(self):
        return self._t.numel()

    @property
    def dtype(self):
        return _dt.from_torch(self._t.dtype)

    @property
    def place(self):
        return place_of(self._t.device)

    @property
    def stop_gradient(self):
        return not self._t.requires_grad

    @stop_gradient.setter
    def stop_gradient(self, v):
        t = self._t
        if v:
            if t.requires_grad:
                self._t = t.detach() if t.grad_fn is not None else t.requires_grad_(False)
        else:
            if not t.requires_grad:
                if t.grad_fn is None and (t.is_floating_point() or t.is_complex()):
                    t.requires_grad_(True)
                elif t.is_floating_point() or t.is_complex():
                    self._t = t.detach().requires_grad_(True)

    @property
    def is_leaf(self):
        return self._t.is_leaf

    @property
    def grad(self):
        g = self._t.grad
        if g is None:
            return None
        if g.dtype != torch.float32 and g.is_floating_point() and self.__dict__.get('_master_grad'):
            return _wrap(g.float())  # amp.decorate(master_grad=True): float32 view of the gradient
        return _wrap(g)

    @grad.setter
    def grad(self, v):
        self._t.grad = None if v is None else _unwrap(v)

    @property
    def data(self):
        return _wrap(self._t.detach())

    @data.setter
    def data(self, v):
        with torch.no_grad():
            self._t.data = _unwrap(v).data if isinstance(v, Tensor) else _as_torch(v, device=self._t.device)

    @property
    def T(self):
        return _wrap(self._t.permute(*reversed(range(self._t.dim()))))

    @property
    def mT(self):
        return _wrap(self._t.transpose(-1, -2))

    @property
    def real(self):
        return _wrap(torch.real(self._t))

    @property
    def imag(self):
        if not self._t.is_complex():  # a real tensor's imaginary part is zero
            return _wrap(torch.zeros_like(self._t))
        return _wrap(torch.imag(self._t))

    @property
    def layout(self):
        return 'NCHW'

    @property
    def strides(self):
        return list(self._t.stride())

    @property
    def offset(self):
        return self._t.storage_offset() * self._t.element_size()

    @property
    def type(self):
        return 'DENSE_TENSOR'

    @property
    def inplace_version(self):
        return self._t._version

    @property
    def is_dist_tensor(self):
        return False

    def is_dense(self):
        return True

    def is_sparse(self):
        return self._t.is_sparse

    def is_sparse_coo(self):
        return self._t.layout == torch.sparse_coo

    def is_sparse_csr(self):
        return self._t.layout == torch.sparse_csr

    def is_contiguous(self):
        return self._t.is_contiguous()

    def contiguous(self):
        return _wrap(self._t.contiguous())

    def element_size(self):
        return self._t.element_size()

    def data_ptr(self):
        return self._t.data_ptr()

    def get_tensor(self):
        return self

    def value(self):
        return self

    def is_floating_point(self):
        return self._t.is_floating_point()

    def is_complex(self):
        return self._t.is_complex()

    def is_integer(self):
        return _dt.is_integer_dtype(self._t.dtype)

    # ------------------------------------------------------------------ conversion
    def numpy(self):
        t = self._t.detach()
        if t.device.type != 'cpu':
            t = t.cpu()
        if t.dtype == torch.bfloat16:
            return t.view(torch.uint16).numpy() if hasattr(torch, 'uint16') else t.float().numpy()
        return t.resolve_conj().numpy()

    def __array__(self, dtype=None, copy=None):
        t = self._t.detach().cpu()
        if t.dtype == torch.bfloat16:
            t = t.float()
        a = t.numpy()
        return a.astype(dtype) if dtype is not None else a

    def tolist(self):
        return self._t.detach().cpu().tolist()

    def item(self, *args):
        if args:
            return self._t.detach()[args].item() if len(args) > 1 else self._t.detach().flatten()[args[0]].item()
        return self._t.item()

    def __float__(self):
        return float(self._t.item())

    def __int__(self):
        return int(self._t.item())

    def __index__(self):
        return int(self._t.item())

    def __bool__(self):
        return bool(self._t.item())

    __nonzero__ = __bool__

    def __len__(self):
        if self._t.dim() == 0:
            raise TypeError("len() of a 0-D tensor")
        return self._t.shape[0]

    def __iter__(self):
        for i in range(len(self)):
            yield _wrap(self._t[i])

    def __hash__(self):
        return id(self)

    def cpu(self):
        return _wrap(self._t.cpu())

    def cuda(self, device_id=None, blocking=True):
        dev = torch.device('cuda', device_id if device_id is not None else (current_device().index or 0))
        return _wrap(self._t.to(dev, non_blocking=not blocking))

    def pin_memory(self, blocking=True):
        return _wrap(self._t.pin_memory())

    def _to(self, device=None, dtype=None, blocking=None):
        t = self._t
        if device is not None:
            t = t.to(to_device(device), non_blocking=blocking is False)
        if dtype is not None:
            t = t.to(_dt.to_torch_dtype(dtype))
        return _wrap(t)

    def to(self, *args, **kwargs):
        device = kwargs.get('device')
        dtype = kwargs.get('dtype')
        blocking = kwargs.get('blocking')
        for a in args:
            if isinstance(a, Tensor):
                device, dtype = a._t.device, a._t.dtype
            elif isinstance(a, (torch.dtype, np.dtype)) or (isinstance(a, str) and a.replace('paddle.', '') in _dt._STR2DTYPE):
                dtype = a
            elif isinstance(a, bool):
                blocking = a
            else:
                device = a
        return self._to(device, dtype, blocking)

    def astype(self, dtype):
        return _wrap(self._t.to(_dt.to_torch_dtype(dtype)))

    cast = astype

    def detach(self):
        return _wrap(self._t.detach())

    def detach_(self):
        self._t = self._t.detach()
        return self

    def clone(self):
        return _wrap(self._t.clone())

    def __copy__(self):
        return _wrap(self._t)

    def __deepcopy__(self, memo):
        new = _wrap(self._t.detach().clone().requires_grad_(self._t.requires_grad))
        new._name = self._name
        new.persistable = self.persistable
        if self.__dict__:
            new.__dict__.update({k: v for k, v in self.__dict__.items()})
        memo[id(self)] = new
        return new

    def __reduce_ex__(self, proto):
        # paddle.save pickles a Tensor as (name, ndarray): framework/io.py reduce_varbase.
        return (tuple, ((self.name, np.asarray(self)),))

    # ------------------------------------------------------------------ autograd
    def backward(self, grad_tensor=None, retain_graph=False):
        g = None if grad_tensor is None else _unwrap(grad_tensor)
        if g is None and self._t.numel() != 1:
            g = torch.ones_like(self._t)
        self._t.backward(g, retain_graph=retain_graph)

    def gradient(self):
        g = self._t.grad
        return None if g is None else _wrap(g).numpy()

    def clear_grad(self, set_to_zero=False):
        if self._t.grad is not None:
            if set_to_zero:
                self._t.grad.zero_()
            else:
                self._t.grad = None

    clear_gradient = clear_grad

    def _clear_data(self):
        self._t = torch.empty(0, dtype=self._t.dtype, device=self._t.device)

    def register_hook(self, hook):
        def h(g):
            r = hook(_wrap(g))
            return None if r is None else _unwrap(r)
        handle = self._t.register_hook(h)
        return handle

    def _register_grad_hook(self, hook):
        return self.register_hook(hook)

    def retain_grads(self):
        self._t.retain_grad()

    # ------------------------------------------------------------------ in-place value ops
    def set_value(self, value):
        v = value._t if isinstance(value, Tensor) else _as_torch(value)
        with torch.no_grad():
            if list(v.shape) != list(self._t.shape):
                raise ValueError(f"set_value shape mismatch {list(v.shape)} vs {self.shape}")
            self._t.copy_(v.to(self._t.dtype))
        return self

    def copy_(self, src, blocking=True):
        with torch.no_grad():
            self._t.copy_(_unwrap(src), non_blocking=not blocking)
        return self

    def zero_(self):
        with torch.no_grad():
            self._t.zero_()
        return self

    def fill_(self, value):
        with torch.no_grad():
            self._t.fill_(value)
        return self

    def apply_(self, func):
        with torch.no_grad():
            self._t.copy_(_unwrap(func(_wrap(self._t.detach()))))
        return self

    def apply(self, func):
        return func(self)

    def _share_buffer_to(self, other):
        other._t = self._t
        return other

    def _is_initialized(self):
        return self._t.numel() > 0 or self._t.dim() > 0

    def _numel(self):
        return self._t.numel()

    # ------------------------------------------------------------------ printing
    def __repr__(self):
        t = self._t.detach()
        body = np.array2string(np.asarray(t.float().cpu() if t.dtype == torch.bfloat16 else t.cpu()),
                               separator=', ', precision=_print_precision(), prefix='       ')
        sg = 'True' if not self._t.requires_grad else 'False'
        return (f"Tensor(shape={self.shape}, dtype={_dt.dtype_name(t.dtype)}, place={self.place}, "
                f"stop_gradient={sg},\n       {body})")

    __str__ = __repr__

    def __format__(self, spec):
        if self._t.dim() == 0:
            return format(self._t.item(), spec)
        return repr(self)


def _print_precision():
    from .printing import _opts
    return _opts['precision']


_PARAMS = weakref.WeakValueDictionary()  # id(storage tensor) -> Parameter (static programs map consts back)


def register_param(p):
    """Re-key a Parameter after its storage tensor was replaced (dtype casts of AMP O2 /
    Layer.to): kernels that accumulate gradients into flat slots look parameters up by tensor."""
    _PARAMS[id(p._t)] = p


class Parameter(Tensor):
    """EagerParamBase: a trainable leaf (reference: python/paddle/base/framework.py EagerParamBase)."""
    __slots__ = ()

    def __init__(self, value, trainable=True, name=None, **kw):
        t = value._t if isinstance(value, Tensor) else (value if isinstance(value, torch.Tensor) else _as_torch(value))
        t = t.detach()
        if trainable and (t.is_floating_point() or t.is_complex()):
            t.requires_grad_(True)
        self._t = t
        self._name = name
        self.persistable = True
        d = self.__dict__
        d['optimize_attr'] = kw.get('optimize_attr', {'learning_rate': 1.0})
        d['regularizer'] = kw.get('regularizer')
        d['do_model_average'] = kw.get('do_model_average')
        d['need_clip'] = kw.get('need_clip', True)
        d['is_distributed'] = kw.get('is_distributed', False)
        d['_trainable'] = trainable
        _PARAMS[id(t)] = self

    @property
    def trainable(self):
        return self.__dict__.get('_trainable', True)

    @trainable.setter
    def trainable(self, v):
        self.__dict__['_trainable'] = v
        self.stop_gradient = not v

    def __repr__(self):
        return 'Parameter containing:\n' + super().__repr__()


EagerParamBase = Parameter


# [True] while a bytecode-translated (jit/sot.py) function runs: the tracer-visible paths below are
# taken only then (a list read instead of torch.compiler.is_compiling() on every wrap)
SOT_ACTIVE = [False]


def _fast_wrap(t, _new=object.__new__, _T=Tensor, _sot=SOT_ACTIVE, _compiling=torch.compiler.is_compiling):
    if _sot[0] and _compiling():  # inside a bytecode translation: a constructor the tracer follows
        return _T(t)
    o = _new(_T)
    o._t = t
    o._name = None
    o.persistable = False
    return o


_wrap = _fast_wrap


def _unwrap(x):
    return x._t if isinstance(x, Tensor) else x


def _as_torch(data, dtype=None, device=None):
    """Convert python/numpy data to a torch tensor with paddle's dtype inference rules."""
    dtype = _dt.to_torch_dtype(dtype)
    if isinstance(data, Tensor):
        t = data._t
    elif isinstance(data, torch.Tensor):
        t = data
    elif isinstance(data, np.ndarray):
        if data.dtype == np.float64 and dtype is None:
            t = torch.from_numpy(np.ascontiguousarray(data))
        elif data.dtype == np.uint16 and dtype in (None, torch.bfloat16):
            t = torch.from_numpy(np.ascontiguousarray(data).view(np.int16)).view(torch.bfloat16)
        elif data.dtype.kind in 'OUS':
            raise TypeError(f"cannot convert numpy array of dtype {data.dtype} to Tensor")
        else:
            t = torch.from_numpy(np.ascontiguousarray(data))
    elif isinstance(data, (bool, np.bool_)):
        t = torch.tensor(bool(data))
    elif isinstance(data, (int, np.integer)):
        t = torch.tensor(int(data), dtype=torch.int64)
    elif isinstance(data, (float, np.floating)):
        t = torch.tensor(float(data), dtype=_dt.default_float())
    elif isinstance(data, complex):
        t = torch.tensor(data, dtype=torch.complex64)
    elif isinstance(data, (list, tuple)):
        if len(data) and any(isinstance(e, Tensor) for e in _flatten_seq(data)):
            t = torch.stack([_as_torch(e) for e in data]) if len(data) else torch.tensor([])
        else:
            arr = np.array(data)
            if arr.dtype == np.float64:
                arr = arr.astype(_dt.to_numpy_dtype(_dt.default_float()) if _dt.default_float() != torch.bfloat16 else np.float32)
            t = torch.from_numpy(arr) if arr.dtype.kind not in 'OUS' else torch.tensor(data)
    else:
        t = torch.as_tensor(data)
    if dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if device is not None and t.device != device:
        t = t.to(device)
    return t


def _flatten_seq(x):
    for e in x:
        if isinstance(e, (list, tuple)):
            yield from _flatten_seq(e)
        else:
            yield e


def to_tensor(data, dtype=None, place=None, stop_gradient=True):
    """paddle.to_tensor (reference: python/paddle/tensor/creation.py to_tensor)."""
    dev = to_device(place)
    if isinstance(data, Tensor):
        t = data._t.detach()
        if dtype is not None:
            t = t.to(_dt.to_torch_dtype(dtype))
        t = t.to(dev).clone() if t.device == dev else t.to(dev)
    else:
        t = _as_torch(data, dtype=dtype, device=dev)
        if isinstance(data, torch.Tensor):
            t = t.detach().clone() if t is data else t
    if not stop_gradient and (t.is_floating_point() or t.is_complex()):
        t = t.requires_grad_(True)
    return _wrap(t)


def is_tensor(x):
    return isinstance(x, Tensor)
