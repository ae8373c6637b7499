"""Data types.

``paddle.float32`` … are :class:`DataType` objects (``paddle.dtype``) that print as
``paddle.float32`` and compare / hash equal to the storage layer's torch dtype, so they key the
same dicts and pass every ``==`` test a torch dtype does; strings (``'float32'``) and numpy dtypes
are accepted everywhere a dtype is taken and normalised by :func:`to_torch_dtype`
(reference: python/paddle/framework/dtype.py, python/paddle/base/data_feeder.py:convert_dtype).
``Tensor.dtype`` returns the DataType; kernels and internal code work on torch dtypes.
"""
import builtins

import numpy as np
import torch

_T = {
    'uint8': torch.uint8, 'int8': torch.int8, 'int16': torch.int16, 'int32': torch.int32, 'int64': torch.int64,
    'float16': torch.float16, 'float32': torch.float32, 'float64': torch.float64, 'bfloat16': torch.bfloat16,
    'bool': torch.bool, 'complex64': torch.complex64, 'complex128': torch.complex128,
    'float8_e4m3fn': torch.float8_e4m3fn, 'float8_e5m2': torch.float8_e5m2,
}


class DataType:
    """A paddle data type: prints ``paddle.<name>``, equals (and hashes as) its torch dtype,
    forwards torch dtype attributes (``is_floating_point``, ``itemsize``, ``is_complex`` ...)."""
    __slots__ = ('_t', 'name')

    def __init__(self, t, name):
        object.__setattr__(self, '_t', t)
        object.__setattr__(self, 'name', name)

    def __repr__(self):
        return f'paddle.{self.name}'

    __str__ = __repr__

    def __eq__(self, other):
        if isinstance(other, DataType):
            return self._t is other._t
        if isinstance(other, torch.dtype):
            return self._t == other
        return False

    def __ne__(self, other):
        return not self.__eq__(other)

    def __hash__(self):
        return hash(self._t)

    def __getattr__(self, k):
        return getattr(object.__getattribute__(self, '_t'), k)

    def __setattr__(self, k, v):
        raise AttributeError('paddle dtypes are immutable')

    def __reduce__(self):
        return (_by_name, (self.name,))

    @property
    def torch_dtype(self):
        return self._t


_D = {n: DataType(t, n) for n, t in _T.items()}
_T2D = {t: d for d, t in ((d, d._t) for d in _D.values())}


def _by_name(name):
    return _D[name]


def from_torch(t):
    """The paddle DataType of a torch dtype (the torch dtype itself for ones paddle has no name for)."""
    return _T2D.get(t, t)


uint8 = _D['uint8']
int8 = _D['int8']
int16 = _D['int16']
int32 = _D['int32']
int64 = _D['int64']
float16 = _D['float16']
half = float16
float32 = _D['float32']
float64 = _D['float64']
bfloat16 = _D['bfloat16']
bool = _D['bool']  # noqa: A001 (paddle.bool)
complex64 = _D['complex64']
complex128 = _D['complex128']
float8_e4m3fn = _D['float8_e4m3fn']
float8_e5m2 = _D['float8_e5m2']

dtype = DataType

_STR2DTYPE = {
    'uint8': _T['uint8'], 'int8': _T['int8'], 'int16': _T['int16'], 'int32': _T['int32'], 'int64': _T['int64'],
    'float16': _T['float16'], 'half': _T['float16'], 'fp16': _T['float16'],
    'float32': _T['float32'], 'float': _T['float32'], 'fp32': _T['float32'],
    'float64': _T['float64'], 'double': _T['float64'], 'fp64': _T['float64'],
    'bfloat16': _T['bfloat16'], 'bf16': _T['bfloat16'], 'uint16': _T['bfloat16'],  # paddle stores bf16 as uint16 in numpy
    'bool': _T['bool'], 'complex64': _T['complex64'], 'complex128': _T['complex128'],
    'float8_e4m3fn': _T['float8_e4m3fn'], 'float8_e5m2': _T['float8_e5m2'],
    'int': _T['int64'], 'long': _T['int64'],
}

_DTYPE2STR = {v: k for k, v in reversed(list(_STR2DTYPE.items()))}
_DTYPE2STR.update({t: n for n, t in _T.items()})

_NP2DTYPE = {
    np.dtype('uint8'): _T['uint8'], np.dtype('int8'): _T['int8'], np.dtype('int16'): _T['int16'],
    np.dtype('int32'): _T['int32'], np.dtype('int64'): _T['int64'], np.dtype('float16'): _T['float16'],
    np.dtype('float32'): _T['float32'], np.dtype('float64'): _T['float64'], np.dtype('bool'): _T['bool'],
    np.dtype('complex64'): _T['complex64'], np.dtype('complex128'): _T['complex128'],
}

_default_dtype = torch.float32


def to_torch_dtype(d):
    """Normalise any paddle-accepted dtype spelling to a torch dtype (None passes through)."""
    if d is None or isinstance(d, torch.dtype):
        return d
    if isinstance(d, DataType):
        return d._t
    if isinstance(d, str):
        r = _STR2DTYPE.get(d.replace('paddle.', ''))
        if r is None:
            raise TypeError(f"unsupported dtype {d!r}")
        return r
    if d is float:
        return torch.float32
    if d is int:
        return torch.int64
    if d is builtins.bool:
        return torch.bool
    try:
        return _NP2DTYPE[np.dtype(d)]
    except Exception:  # pragma: no cover
        raise TypeError(f"unsupported dtype {d!r}")


def dtype_name(d):
    if isinstance(d, DataType):
        return d.name
    return _DTYPE2STR.get(d, str(d).replace('torch.', ''))


def to_numpy_dtype(d):
    d = to_torch_dtype(d)
    if d == torch.bfloat16:
        return np.dtype('uint16')
    return torch.empty((), dtype=d).numpy().dtype


def set_default_dtype(d):
    global _default_dtype
    d = to_torch_dtype(d)
    if d not in (torch.float16, torch.float32, torch.float64, torch.bfloat16):
        raise TypeError("set_default_dtype only supports float16/float32/float64/bfloat16")
    _default_dtype = d
    torch.set_default_dtype(d if d in (torch.float32, torch.float64) else torch.float32)


def get_default_dtype():
    return dtype_name(_default_dtype)


def default_float():
    return _default_dtype


def is_floating(d):
    return to_torch_dtype(d).is_floating_point


def is_complex_dtype(d):
    return to_torch_dtype(d).is_complex


def is_integer_dtype(d):
    d = to_torch_dtype(d)
    return not d.is_floating_point and not d.is_complex and d != torch.bool


class finfo:
    """paddle.finfo (reference: python/paddle/framework/dtype.py)."""

    def __init__(self, d):
        i = torch.finfo(to_torch_dtype(d))
        self.dtype = dtype_name(to_torch_dtype(d))
        self.bits, self.eps, self.max, self.min = i.bits, i.eps, i.max, i.min
        self.tiny = self.smallest_normal = i.tiny
        self.resolution = i.resolution

    def __repr__(self):
        return f"finfo(min={self.min}, max={self.max}, eps={self.eps}, dtype={self.dtype})"


class iinfo:
    def __init__(self, d):
        i = torch.iinfo(to_torch_dtype(d))
        self.dtype = dtype_name(to_torch_dtype(d))
        self.bits, self.max, self.min = i.bits, i.max, i.min

    def __repr__(self):
        return f"iinfo(min={self.min}, max={self.max}, bits={self.bits}, dtype={self.dtype})"
