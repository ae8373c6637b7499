"""paddle.framework (reference: python/paddle/framework/__init__.py, base/framework.py)."""
import os

import numpy as np
import torch

from .param_attr import ParamAttr, WeightNormParamAttr  # noqa: F401
from .io import save, load, async_save  # noqa: F401
from . import flags as _flags
from .flags import set_flags, get_flags  # noqa: F401

_static_mode = [False]


def in_dynamic_mode():
    return not _static_mode[0]


in_dygraph_mode = in_dynamic_mode


def in_pir_mode():
    return _static_mode[0]


def enable_static():
    _static_mode[0] = True
    from ..static.program import _start_recording
    _start_recording()


def disable_static(place=None):
    _static_mode[0] = False
    from ..static.program import _stop_recording
    _stop_recording()
    if place is not None:
        from ..core.place import set_device
        set_device(place)


def seed(s):
    """paddle.seed: seeds the host and every HIP device generator."""
    import random
    random.seed(s)
    np.random.seed(s % (2 ** 32))
    torch.manual_seed(s)
    from ..core.tensor import _wrap
    return torch.default_generator


def _host_seed():
    """A 63-bit seed drawn from the global (paddle.seed-controlled) host generator."""
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def get_rng_state(device=None):
    from ..core.tensor import _wrap
    st = [_wrap(torch.get_rng_state())]
    if torch.cuda.is_available():
        st += [_wrap(s) for s in torch.cuda.get_rng_state_all()]
    return st


def set_rng_state(state_list, device=None):
    from ..core.tensor import _unwrap
    torch.set_rng_state(_unwrap(state_list[0]).cpu())
    if torch.cuda.is_available() and len(state_list) > 1:
        torch.cuda.set_rng_state_all([_unwrap(s).cpu() for s in state_list[1:]])


def get_cuda_rng_state():
    from ..core.tensor import _wrap
    return [_wrap(s) for s in torch.cuda.get_rng_state_all()] if torch.cuda.is_available() else []


def set_cuda_rng_state(state_list):
    from ..core.tensor import _unwrap
    if torch.cuda.is_available():
        torch.cuda.set_rng_state_all([_unwrap(s).cpu() for s in state_list])


class LazyGuard:
    """paddle.LazyGuard: parameters created inside are materialised lazily (here: eagerly on the
    current device; MI355X HBM (288 GB) holds even 13B models unsharded for init)."""

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _current_expected_place():
    from ..core.place import current_device, place_of
    return place_of(current_device())


_ = os

from .. import core  # noqa: E402,F401  (paddle.framework.core: reference C++ module surface)
