"""Hand-written HIP/CDNA4 operator library (python side).

``use_hip(t)`` decides whether a tensor takes the native kernel path: it is True for every
tensor on the GPU.  If the kernel library is missing on a GPU process it raises instead of
silently falling back (``PADDLE_AMD_DISABLE_HIP_KERNELS=1`` opts out explicitly, for A/B).
"""
from ..framework.flags import pa_flag  # noqa: E402
import os

import torch

from . import _native
from ..core.tensor import SOT_ACTIVE as _SOT

_disabled = pa_flag('disable_hip_kernels')


def enabled():
    return not _disabled


def set_enabled(v):
    global _disabled
    _disabled = not v


def use_hip(t, _compiling=torch.compiler.is_compiling):
    if _disabled or not isinstance(t, torch.Tensor) or t.device.type != 'cuda':
        return False
    if _SOT[0] and _compiling():  # bytecode translation (jit/sot.py): torch composites, mapped back by the Executor
        return False
    if _native.lib is None and _native._load() is None:
        raise RuntimeError("paddle_amd HIP kernel library not available on a GPU process: " + str(_native.load_error))
    return True


def native_loaded():
    return _native.lib is not None


from . import norm, softmax, act, xent, embedding, rope, optim, flash_attn, gemm, linear, fused, batchnorm, conv, pool  # noqa: E402,F401,E501
from . import decode  # noqa: E402,F401
from . import fp8  # noqa: E402,F401
from . import matmul  # noqa: E402,F401
from . import woq  # noqa: E402,F401
from . import int8  # noqa: E402,F401
