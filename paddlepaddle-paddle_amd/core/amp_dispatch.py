"""Per-op AMP dispatch: the dygraph tracer's auto-cast rule, applied at the paddle op boundary.

Reference: paddle/fluid/eager/amp_utils.h (``GetAmpDestDtype`` / ``GetPromoteType``) and
paddle/fluid/imperative/amp_auto_cast.cc, driven by python/paddle/amp/auto_cast.py:383
(``amp_guard``) with the op lists of python/paddle/amp/amp_lists.py.

Every public op that appears in a reference AMP list is tagged with its reference op name
(``@amp_op('matmul_v2')``).  Inside an active ``amp_guard`` the wrapper decides the op's
destination dtype and casts its floating inputs (Tensors, and Tensors inside list/tuple
arguments) before the op runs:

* op in the black list            -> float32
* op in the white list            -> the AMP dtype (float16 / bfloat16)
* otherwise (gray)                -> no cast: mixed inputs promote to the wider type
  (``use_promote=True`` semantics — the reference default)

Level O1 uses the full black list; O2 only the "extra" black list (interp / lookup_table /
scatter), so in O2 softmax / layer_norm / losses run in the low-precision dtype like the
reference's pure-fp16 mode; OD keeps only the white list.  The wrapper's fast path when AMP is
off is one attribute test.
"""
import functools

import torch

_LOW = (torch.float16, torch.bfloat16)


class _AmpState:
    __slots__ = ('active', 'level', 'dtype', 'white', 'black', 'use_promote', 'ops_seen', 'post')

    def __init__(self):
        self.active = False
        self.level = 'O0'
        self.dtype = torch.float16
        self.white = frozenset()
        self.black = frozenset()
        self.use_promote = True
        self.ops_seen = None  # dict op -> {dtype name: count} while collect_operator_stats runs
        self.post = None  # callable(op, output) while the tensor checker dumps op outputs


STATE = _AmpState()


def dest_dtype(op):
    """Destination dtype of ``op`` under the current AMP state (None: leave inputs alone)."""
    st = STATE
    if not st.active:
        return None
    if op in st.black:
        return torch.float32
    if op in st.white:
        return st.dtype
    return None


def _cast(a, dst):
    from .tensor import Tensor, _wrap
    if isinstance(a, Tensor):
        t = a._t
        if t.dtype != dst and (t.dtype in _LOW or t.dtype == torch.float32):
            return _wrap(t.to(dst))
        return a
    if isinstance(a, (list, tuple)) and a and any(isinstance(e, Tensor) for e in a):
        return type(a)(_cast(e, dst) for e in a)
    return a


def _record(op, args):
    from .tensor import Tensor
    dt = None
    for a in args:
        if isinstance(a, Tensor) and a._t.is_floating_point():
            dt = a._t.dtype
            break
    name = {torch.float32: 'float32', torch.float16: 'float16', torch.bfloat16: 'bfloat16'}.get(dt, 'other')
    d = STATE.ops_seen.setdefault(op, {})
    d[name] = d.get(name, 0) + 1


def amp_op(op):
    """Tag a public op with its reference AMP op name and apply the auto-cast rule to it."""
    def deco(fn):
        @functools.wraps(fn)
        def wrapper(*args, **kwargs):
            st = STATE
            if not st.active and st.ops_seen is None and st.post is None:
                return fn(*args, **kwargs)
            dst = dest_dtype(op)
            if dst is not None:
                args = tuple(_cast(a, dst) for a in args)
                if kwargs:
                    kwargs = {k: _cast(v, dst) for k, v in kwargs.items()}
            if st.ops_seen is not None:
                _record(op, args)
            out = fn(*args, **kwargs)
            if st.post is not None:
                st.post(op, out)
            return out
        wrapper._amp_op = op
        return wrapper
    return deco


def wrap(fn, op):
    return amp_op(op)(fn)
