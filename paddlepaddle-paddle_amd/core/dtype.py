"""Data types.

Paddle exposes ``paddle.float32`` … as ``paddle.dtype`` values and accepts strings
(``'float32'``) and numpy dtypes everywhere a dtype is taken
(reference: python/paddle/framework/dtype.py, python/paddle/base/data_feeder.py:convert_dtype).
Here the dtype objects ARE the torch dtypes of the storage layer, so no translation
happens on the hot path; strings / numpy dtypes are normalised by :func:`to_torch_dtype`.
"""
import builtins

import numpy as np
import torch

uint8 = torch.uint8
int8 = torch.int8
int16 = torch.int16
int32 = torch.int32
int64 = torch.int64
float16 = torch.float16
half = torch.float16
float32 = torch.float32
float64 = torch.float64
bfloat16 = torch.bfloat16
bool = torch.bool  # noqa: A001 (paddle.bool)
complex64 = torch.complex64
complex128 = torch.complex128
float8_e4m3fn = torch.float8_e4m3fn
float8_e5m2 = torch.float8_e5m2

dtype = torch.dtype

_STR2DTYPE = {
    'uint8': uint8, 'int8': int8, 'int16': int16, 'int32': int32, 'int64': int64,
    'float16': float16, 'half': float16, 'fp16': float16,
    'float32': float32, 'float': float32, 'fp32': float32,
    'float64': float64, 'double': float64, 'fp64': float64,
    'bfloat16': bfloat16, 'bf16': bfloat16, 'uint16': bfloat16,  # paddle stores bf16 as uint16 in numpy
    'bool': bool, 'complex64': complex64, 'complex128': complex128,
    'float8_e4m3fn': float8_e4m3fn, 'float8_e5m2': float8_e5m2,
    'int': int64, 'long': int64,
}

_DTYPE2STR = {v: k for k, v in reversed(list(_STR2DTYPE.items()))}
_DTYPE2STR.update({float32: 'float32', float16: 'float16', float64: 'float64', bfloat16: 'bfloat16',
                   int64: 'int64', int32: 'int32', bool: 'bool'})

_NP2DTYPE = {
    np.dtype('uint8'): uint8, np.dtype('int8'): int8, np.dtype('int16'): int16,
    np.dtype('int32'): int32, np.dtype('int64'): int64, np.dtype('float16'): float16,
    np.dtype('float32'): float32, np.dtype('float64'): float64, np.dtype('bool'): bool,
    np.dtype('complex64'): complex64, np.dtype('complex128'): complex128,
}

_default_dtype = float32


def to_torch_dtype(d):
    """Normalise any paddle-accepted dtype spelling to a torch dtype (None passes through)."""
    if d is None or isinstance(d, torch.dtype):
        return d
    if isinstance(d, str):
        r = _STR2DTYPE.get(d.replace('paddle.', ''))
        if r is None:
            raise TypeError(f"unsupported dtype {d!r}")
        return r
    if d is float:
        return float32
    if d is int:
        return int64
    if d is builtins.bool:
        return bool
    try:
        return _NP2DTYPE[np.dtype(d)]
    except Exception:  # pragma: no cover
        raise TypeError(f"unsupported dtype {d!r}")


def dtype_name(d):
    return _DTYPE2STR.get(d, str(d).replace('torch.', ''))


def to_numpy_dtype(d):
    d = to_torch_dtype(d)
    if d == bfloat16:
        return np.dtype('uint16')
    return torch.empty((), dtype=d).numpy().dtype


def set_default_dtype(d):
    global _default_dtype
    d = to_torch_dtype(d)
    if d not in (float16, float32, float64, bfloat16):
        raise TypeError("set_default_dtype only supports float16/float32/float64/bfloat16")
    _default_dtype = d
    torch.set_default_dtype(d if d in (float32, float64) else float32)


def get_default_dtype():
    return dtype_name(_default_dtype)


def default_float():
    return _default_dtype


def is_floating(d):
    return d.is_floating_point


def is_complex_dtype(d):
    return d.is_complex


def is_integer_dtype(d):
    return not d.is_floating_point and not d.is_complex and d != bool


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
