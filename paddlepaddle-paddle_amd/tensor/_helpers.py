"""Shared argument normalisation for the tensor API (paddle axis/shape conventions)."""
import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap, _as_torch  # noqa: F401
from ..core import dtype as _dt

_w = _wrap
_u = _unwrap


def _t(x, like=None):
    """Unwrap to torch; python scalars/ndarrays become tensors on ``like``'s device."""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    dev = like.device if isinstance(like, torch.Tensor) else None
    if isinstance(x, np.ndarray) or isinstance(x, (list, tuple)):
        return _as_torch(x, device=dev)
    return x


def _axis(axis):
    """paddle axis (None/int/list/tuple/Tensor) → None | int | tuple."""
    if axis is None:
        return None
    if isinstance(axis, Tensor):
        axis = axis._t.tolist()
    if isinstance(axis, (list, tuple)):
        if len(axis) == 0:
            return None
        return tuple(int(a) for a in axis)
    return int(axis)


def _dims(axis, ndim):
    """axis → tuple of dims for reductions ('None' = all)."""
    a = _axis(axis)
    if a is None:
        return tuple(range(ndim))
    if isinstance(a, int):
        return (a,)
    return a


def _shape(shape):
    """paddle shape (list of int/Tensor, tuple, Tensor) → list[int]."""
    if isinstance(shape, Tensor):
        return [int(v) for v in shape._t.reshape(-1).tolist()]
    if isinstance(shape, torch.Tensor):
        return [int(v) for v in shape.reshape(-1).tolist()]
    if isinstance(shape, (int, np.integer)):
        return [int(shape)]
    return [int(s._t.item()) if isinstance(s, Tensor) else int(s) for s in shape]


def _scalar(v):
    if isinstance(v, Tensor):
        return v._t.item() if v._t.numel() == 1 else v._t
    return v


def _dtype(d):
    return _dt.to_torch_dtype(d)


def _inplace(x, t):
    """Finish an in-place paddle op: storage already mutated, return the handle."""
    return x
