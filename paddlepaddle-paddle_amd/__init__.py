"""paddle — an MI355X-native deep-learning framework with PaddlePaddle's Python API.

Importable as ``paddle`` (see /paddle/__init__.py at the repository root).  Layout:

* ``core/``      Tensor handle over HIP storage, dtypes, places, method/operator binding
* ``tensor/``    the ``paddle.*`` tensor API
* ``nn/``        Layer, layers, functional, initializers, clipping
* ``ops/``       hand-written HIP/CDNA4 kernel library bindings (csrc/*.hip)
* ``optimizer/`` optimizers + LR schedulers (fused flat-buffer AdamW on GPU)
* ``parallel/``  MI355X engines: flat buffers, bucketed RCCL DP, sharding, TP/SP/PP
* ``distributed/`` paddle.distributed + fleet API on top of ``parallel/``
* ``models/``    GPT / Llama / ERNIE model zoo used by benchmarks
* ``static/``, ``jit/``, ``io/``, ``amp/``, ``vision/``, ``hapi/``, ``profiler/`` …

Reference: python/paddle/__init__.py.
"""
import importlib as _importlib

__version__ = '3.0.0-mi355x'
version = type('version', (), {'full_version': __version__, 'major': '3', 'minor': '0', 'patch': '0',
                                'rc': '0', 'cuda': lambda: 'False', 'cudnn': lambda: 'False',
                                'rocm': lambda: '7.2', 'show': staticmethod(lambda: print(__version__))})

from .core import dtype as _dtype_mod  # noqa: E402
from .core.dtype import (uint8, int8, int16, int32, int64, float16, float32, float64, bfloat16, bool,  # noqa: E402,F401,A004
                         complex64, complex128, float8_e4m3fn, float8_e5m2, dtype, finfo, iinfo,
                         set_default_dtype, get_default_dtype)
from .core.place import (CPUPlace, CUDAPlace, CUDAPinnedPlace, XPUPlace, CustomPlace, IPUPlace, Place,  # noqa: E402,F401
                         set_device, get_device, is_compiled_with_cuda, is_compiled_with_rocm,
                         is_compiled_with_xpu, is_compiled_with_custom_device, is_compiled_with_distribute,
                         is_compiled_with_cinn)
from .core.tensor import Tensor, Parameter, to_tensor, is_tensor  # noqa: E402,F401
from . import tensor  # noqa: E402,F401
from .tensor import all_functions as _all_functions  # noqa: E402

_ns = _all_functions()
globals().update({k: v for k, v in _ns.items() if k not in ('Tensor',)})

from .core import tensor_methods as _tm  # noqa: E402
_tm.install(_ns)

from .autograd import no_grad, enable_grad, set_grad_enabled, is_grad_enabled, grad, PyLayer  # noqa: E402,F401
from . import autograd  # noqa: E402,F401
from .framework import (ParamAttr, WeightNormParamAttr, save, load, async_save, set_flags, get_flags,  # noqa: E402,F401
                        in_dynamic_mode, in_dygraph_mode, enable_static, disable_static, seed, get_rng_state,
                        set_rng_state, get_cuda_rng_state, set_cuda_rng_state, LazyGuard)
from . import framework  # noqa: E402,F401
from . import nn  # noqa: E402,F401
from . import optimizer  # noqa: E402,F401
from . import regularizer  # noqa: E402,F401
from . import ops  # noqa: E402,F401
from . import _C_ops  # noqa: E402,F401
from . import pir  # noqa: E402,F401
from .tensor.linalg import (matmul, bmm, mm, dot, mv, einsum, norm as _norm, cdist, pdist, histogram,  # noqa: E402,F401
                            histogramdd, bincount, cross)
from .tensor.math import prod  # noqa: E402,F401

create_parameter = _ns['create_parameter']

_LAZY = {
    'io': '.io', 'amp': '.amp', 'device': '.device', 'distributed': '.distributed', 'static': '.static',
    'jit': '.jit', 'vision': '.vision', 'metric': '.metric', 'hapi': '.hapi', 'profiler': '.profiler',
    'incubate': '.incubate', 'models': '.models', 'parallel': '.parallel', 'utils': '.utils',
    'linalg': '.linalg', 'fft': '.fft', 'signal': '.signal', 'distribution': '.distribution',
    'sparse': '.sparse', 'text': '.text', 'audio': '.audio', 'geometric': '.geometric',
    'quantization': '.quantization', 'inference': '.inference', 'callbacks': '.hapi.callbacks',
    'onnx': '.onnx', 'sysconfig': '.sysconfig', 'base': '.base', 'decomposition': '.decomposition',
    'hub': '.hapi.hub', 'reader': '.reader', 'dataset': '.dataset', 'cost_model': '.cost_model',
    'cuda': '.device.cuda',
}
_LAZY_ATTR = {
    'Model': ('.hapi', 'Model'), 'summary': ('.hapi', 'summary'), 'flops': ('.hapi', 'flops'),
    'DataParallel': ('.distributed', 'DataParallel'), 'set_printoptions': ('.core.printing', 'set_printoptions'),
    'disable_signal_handler': ('.utils', 'disable_signal_handler'), 'get_cudnn_version': ('.device', 'get_cudnn_version'),
    'check_shape': ('.utils', 'check_shape'), 'batch': ('.io.batch', 'batch'), 'grad_fn': ('.autograd', 'grad'), 'iinfo': ('.core.dtype', 'iinfo'),
}


def __getattr__(name):
    if name in _LAZY:
        mod = _importlib.import_module(_LAZY[name], __name__)
        globals()[name] = mod
        return mod
    if name in _LAZY_ATTR:
        m, a = _LAZY_ATTR[name]
        v = getattr(_importlib.import_module(m, __name__), a)
        globals()[name] = v
        return v
    raise AttributeError(f"module 'paddle' has no attribute '{name}'")


def in_cinn_mode():
    return False


def is_compiled_with_ipu():
    return False


def get_all_custom_device_type():
    return []


def _maybe_native_allocator():
    """FLAGS_use_native_allocator=1: install csrc/alloc's auto-growth best-fit allocator as the
    device allocator before anything allocates on the GPU."""
    import os as _os
    if _os.environ.get('FLAGS_use_native_allocator', '').lower() in ('1', 'true', 'yes', 'on'):
        from .device.cuda import allocator as _native_alloc
        _native_alloc.enable()


_maybe_native_allocator()
