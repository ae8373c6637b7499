"""paddle.base.core / paddle.framework.core — the names third-party Paddle code reaches for on the
reference's C++ extension module (reference: python/paddle/base/core.py, the pybind module
paddle/fluid/pybind/pybind.cc): ``core.eager.Tensor``, ``core.VarDesc.VarType`` / ``core.DataType``
dtype enums, the ``is_compiled_with_*`` probes, places, ``globals()`` (the flag registry), the
prim switches, generators.  Everything maps onto this framework's own modules (the tensor layer,
framework/flags.py, the HIP device); submodules (tensor, dtype, place, ...) import lazily."""
import enum as _enum

from .place import (is_compiled_with_cuda, is_compiled_with_rocm, is_compiled_with_xpu,  # noqa: F401
                    is_compiled_with_custom_device, is_compiled_with_distribute, is_compiled_with_cinn,
                    CPUPlace, CUDAPlace, CUDAPinnedPlace)


def is_compiled_with_ipu():
    return False


def is_compiled_with_mkldnn():
    return False


def is_compiled_with_nccl():
    return True  # RCCL, torch.distributed's 'nccl' backend on ROCm


def get_cuda_device_count():
    import torch
    return torch.cuda.device_count()


get_device_count = get_cuda_device_count


class _VarType(_enum.IntEnum):
    """framework.proto VarType.Type codes (the values the reference's ProgramDesc carries)."""
    BOOL = 0
    INT16 = 1
    INT32 = 2
    INT64 = 3
    FP16 = 4
    FP32 = 5
    FP64 = 6
    LOD_TENSOR = 7
    SELECTED_ROWS = 8
    FEED_MINIBATCH = 9
    FETCH_LIST = 10
    STEP_SCOPES = 11
    LOD_RANK_TABLE = 12
    LOD_TENSOR_ARRAY = 13
    PLACE_LIST = 14
    READER = 15
    RAW = 17
    TUPLE = 18
    UINT8 = 20
    INT8 = 21
    BF16 = 22
    COMPLEX64 = 23
    COMPLEX128 = 24
    STRING = 25
    STRINGS = 26
    FP8_E4M3FN = 32
    FP8_E5M2 = 33


class VarDesc:
    VarType = _VarType


class DataType(_enum.IntEnum):
    """phi::DataType (PIR dtype enum)."""
    UNDEFINED = 0
    BOOL = 1
    UINT8 = 2
    INT8 = 3
    UINT16 = 4
    INT16 = 5
    UINT32 = 6
    INT32 = 7
    UINT64 = 8
    INT64 = 9
    FLOAT32 = 10
    FLOAT64 = 11
    COMPLEX64 = 12
    COMPLEX128 = 13
    FLOAT16 = 15
    BFLOAT16 = 16
    FLOAT8_E4M3FN = 18
    FLOAT8_E5M2 = 19


class _Eager:
    """core.eager: the eager Tensor type (this framework's paddle.Tensor)."""

    @property
    def Tensor(self):  # noqa: N802
        from .tensor import Tensor
        return Tensor

    TensorBase = Tensor

    @property
    def ops(self):
        from .. import _C_ops
        return _C_ops


eager = _Eager()


def globals():  # noqa: A001 — reference name
    """The FLAGS_* registry as a mutable mapping (core.globals()['FLAGS_x'] = v)."""
    from ..framework import flags as _f
    return _f._FlagsView()


def _set_prim_all_enabled(v):
    from ..framework import flags as _f
    _f.set_flags({'FLAGS_prim_all': bool(v)})


def _set_prim_forward_enabled(v):
    from ..framework import flags as _f
    _f.set_flags({'FLAGS_prim_forward': bool(v)})


def _set_prim_backward_enabled(v):
    from ..framework import flags as _f
    _f.set_flags({'FLAGS_prim_backward': bool(v)})


def _is_fwd_prim_enabled():
    from ..framework import flags as _f
    return bool(_f.get_flags(['FLAGS_prim_forward']).get('FLAGS_prim_forward', False))


def _is_bwd_prim_enabled():
    from ..framework import flags as _f
    return bool(_f.get_flags(['FLAGS_prim_backward']).get('FLAGS_prim_backward', False))


def _is_all_prim_enabled():
    from ..framework import flags as _f
    return bool(_f.get_flags(['FLAGS_prim_all']).get('FLAGS_prim_all', False))


def default_cpu_generator():
    import torch
    return torch.default_generator


def default_cuda_generator(device_id=0):
    import torch
    return torch.cuda.default_generators[device_id] if torch.cuda.is_available() else torch.default_generator


def Scope():  # noqa: N802
    from ..static import global_scope
    return type(global_scope())()


def DenseTensor():  # noqa: N802
    from .tensor import Tensor
    return Tensor.__new__(Tensor)


LoDTensor = DenseTensor


def set_num_threads(n):
    import torch
    torch.set_num_threads(int(n))


def get_num_threads():
    import torch
    return torch.get_num_threads()


def nvprof_nvtx_push(name):
    import torch
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)


def nvprof_nvtx_pop():
    import torch
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_pop()
