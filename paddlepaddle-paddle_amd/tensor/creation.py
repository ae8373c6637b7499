"""paddle creation API (reference: python/paddle/tensor/creation.py)."""
import numpy as np
import torch

from ._helpers import _w, _u, _shape, _dtype, _scalar, Tensor
from ..core import dtype as _dt
from ..core.place import current_device, to_device
from ..core.tensor import to_tensor, _as_torch  # noqa: F401


def _fdt(dtype):
    return _dtype(dtype) if dtype is not None else _dt.default_float()


def zeros(shape, dtype=None, name=None, device=None):
    return _w(torch.zeros(_shape(shape), dtype=_fdt(dtype), device=to_device(device)))


def ones(shape, dtype=None, name=None, device=None):
    return _w(torch.ones(_shape(shape), dtype=_fdt(dtype), device=to_device(device)))


def empty(shape, dtype=None, name=None, device=None):
    return _w(torch.empty(_shape(shape), dtype=_fdt(dtype), device=to_device(device)))


def full(shape, fill_value, dtype=None, name=None, device=None):
    v = _scalar(fill_value)
    if dtype is None:
        dtype = (torch.bool if isinstance(v, bool) else torch.int64 if isinstance(v, int) else _dt.default_float())
    return _w(torch.full(_shape(shape), v, dtype=_dtype(dtype), device=to_device(device)))


def _like(x, dtype):
    t = _u(x)
    return t, (_dtype(dtype) if dtype is not None else t.dtype)


def zeros_like(x, dtype=None, name=None):
    t, d = _like(x, dtype)
    return _w(torch.zeros_like(t, dtype=d))


def ones_like(x, dtype=None, name=None):
    t, d = _like(x, dtype)
    return _w(torch.ones_like(t, dtype=d))


def empty_like(x, dtype=None, name=None):
    t, d = _like(x, dtype)
    return _w(torch.empty_like(t, dtype=d))


def full_like(x, fill_value, dtype=None, name=None):
    t, d = _like(x, dtype)
    return _w(torch.full_like(t, _scalar(fill_value), dtype=d))


def arange(start=0, end=None, step=1, dtype=None, name=None):
    start, end, step = _scalar(start), _scalar(end), _scalar(step)
    if end is None:
        start, end = 0, start
    if dtype is None:
        dtype = torch.int64 if all(isinstance(v, (int, np.integer)) for v in (start, end, step)) else _dt.default_float()
    return _w(torch.arange(start, end, step, dtype=_dtype(dtype), device=current_device()))


def linspace(start, stop, num, dtype=None, name=None):
    return _w(torch.linspace(_scalar(start), _scalar(stop), int(_scalar(num)), dtype=_fdt(dtype), device=current_device()))


def logspace(start, stop, num, base=10.0, dtype=None, name=None):
    return _w(torch.logspace(_scalar(start), _scalar(stop), int(_scalar(num)), base=_scalar(base), dtype=_fdt(dtype),
                             device=current_device()))


def eye(num_rows, num_columns=None, dtype=None, name=None):
    num_columns = num_rows if num_columns is None else num_columns
    return _w(torch.eye(int(_scalar(num_rows)), int(_scalar(num_columns)), dtype=_fdt(dtype), device=current_device()))


def meshgrid(*args, **kwargs):
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        args = args[0]
    return [_w(g) for g in torch.meshgrid(*[_u(a) for a in args], indexing='ij')]


def diag(x, offset=0, padding_value=0, name=None):
    t = _u(x)
    if t.dim() == 1 and padding_value != 0:
        n = t.numel() + abs(offset)
        out = torch.full((n, n), padding_value, dtype=t.dtype, device=t.device)
        return _w(out + torch.diag(t, offset) - torch.diag(torch.full_like(t, padding_value), offset))
    return _w(torch.diag(t, offset))


def diagflat(x, offset=0, name=None):
    return _w(torch.diagflat(_u(x), offset))


def diag_embed(input, offset=0, dim1=-2, dim2=-1):  # noqa: A002
    return _w(torch.diag_embed(_u(input), offset, dim1, dim2))


def diagonal(x, offset=0, axis1=0, axis2=1, name=None):
    return _w(torch.diagonal(_u(x), offset, axis1, axis2))


def tril(x, diagonal=0, name=None):
    return _w(torch.tril(_u(x), diagonal))


def triu(x, diagonal=0, name=None):
    return _w(torch.triu(_u(x), diagonal))


def tril_(x, diagonal=0, name=None):
    x._t.tril_(diagonal)
    return x


def triu_(x, diagonal=0, name=None):
    x._t.triu_(diagonal)
    return x


def tril_indices(row, col, offset=0, dtype='int64'):
    return _w(torch.tril_indices(row, col, offset, dtype=_dtype(dtype), device=current_device()))


def triu_indices(row, col=None, offset=0, dtype='int64'):
    return _w(torch.triu_indices(row, row if col is None else col, offset, dtype=_dtype(dtype), device=current_device()))


def assign(x, output=None):
    if isinstance(x, Tensor):
        t = x._t.clone()
    else:
        t = _as_torch(np.asarray(x) if isinstance(x, (list, tuple)) else x, device=current_device())
        if t.dtype == torch.float64 and not isinstance(x, np.ndarray):
            t = t.float()
    if output is not None:
        with torch.no_grad():
            output._t.copy_(t)
        return output
    return _w(t)


def clone(x, name=None):
    return _w(_u(x).clone())


def complex(real, imag, name=None):  # noqa: A001
    return _w(torch.complex(_u(real), _u(imag)))


def polar(abs, angle, name=None):  # noqa: A002
    return _w(torch.polar(_u(abs), _u(angle)))


def create_parameter(shape, dtype, name=None, attr=None, is_bias=False, default_initializer=None):
    from ..nn.layer.layers import _create_parameter
    return _create_parameter(_shape(shape), dtype, attr=attr, is_bias=is_bias, default_initializer=default_initializer,
                             name=name)


def create_tensor(dtype, name=None, persistable=False):
    return _w(torch.empty(0, dtype=_dtype(dtype), device=current_device()))


def fill_constant(shape, dtype, value, force_cpu=False, out=None, name=None):
    r = full(shape, value, dtype)
    if out is not None:
        out._t = r._t
        return out
    return r
