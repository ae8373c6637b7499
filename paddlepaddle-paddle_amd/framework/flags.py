"""Global FLAGS registry (reference: paddle/common/flags.cc, python paddle.set_flags/get_flags).

Flags are typed, default-valued, overridable from the environment (``FLAGS_xxx=...``) and
readable/settable at run time.  Flags that change framework behaviour here:
``FLAGS_check_nan_inf`` (op-output NaN/Inf checker, amp/debugging.py),
``FLAGS_use_hip_kernels`` (route hot ops to the HIP kernel library),
``FLAGS_allocator_strategy`` / ``FLAGS_fraction_of_gpu_memory_to_use`` (caching allocator knobs),
``FLAGS_use_native_allocator`` / ``FLAGS_auto_growth_chunk_size_in_mb`` (install the native
auto-growth best-fit device allocator, device/cuda/allocator.py, at import).
"""
import os

_REGISTRY = {
    'FLAGS_check_nan_inf': False,
    'FLAGS_check_nan_inf_level': 0,
    'FLAGS_use_hip_kernels': True,
    'FLAGS_allocator_strategy': 'auto_growth',
    'FLAGS_fraction_of_gpu_memory_to_use': 0.92,
    'FLAGS_use_native_allocator': False,
    'FLAGS_auto_growth_chunk_size_in_mb': 0,
    'FLAGS_eager_delete_tensor_gb': 0.0,
    'FLAGS_cudnn_deterministic': False,
    'FLAGS_embedding_deterministic': 0,
    'FLAGS_enable_pir_api': False,
    'FLAGS_use_cuda_graph': False,
    'FLAGS_conv_workspace_size_limit': 512,
    'FLAGS_cudnn_exhaustive_search': False,
    'FLAGS_benchmark': False,
    'FLAGS_call_stack_level': 1,
    'FLAGS_selected_gpus': '0',
    'FLAGS_comm_timeout_seconds': 1800,
    'FLAGS_enable_async_trace': False,
    'FLAGS_prim_all': False,
    'FLAGS_prim_forward': False,
    'FLAGS_prim_backward': False,
}


def _parse(default, s):
    if isinstance(default, bool):
        return s.lower() in ('1', 'true', 'yes', 'on')
    if isinstance(default, int):
        return int(s)
    if isinstance(default, float):
        return float(s)
    return s


for _k, _v in list(_REGISTRY.items()):
    if _k in os.environ:
        try:
            _REGISTRY[_k] = _parse(_v, os.environ[_k])
        except ValueError:
            pass

_hooks = {}


def on_change(name, fn):
    _hooks.setdefault(name, []).append(fn)


def set_flags(flags):
    if not isinstance(flags, dict):
        raise TypeError("flags in set_flags should be a dict")
    for k, v in flags.items():
        if not k.startswith('FLAGS_'):
            k = 'FLAGS_' + k
        if k not in _REGISTRY:
            raise ValueError(f"Flag {k} cannot set its value through this function.")
        _REGISTRY[k] = v
        for fn in _hooks.get(k, []):
            fn(v)


def get_flags(flags):
    if isinstance(flags, str):
        flags = [flags]
    out = {}
    for k in flags:
        kk = k if k.startswith('FLAGS_') else 'FLAGS_' + k
        if kk not in _REGISTRY:
            raise ValueError(f"Flag {k} is not registered")
        out[k] = _REGISTRY[kk]
    return out


def get(name, default=None):
    return _REGISTRY.get(name, default)


class _FlagsView:
    """core.globals(): dict-style access to the registry (setting goes through set_flags)."""

    def __getitem__(self, k):
        return get_flags([k])[k]

    def __setitem__(self, k, v):
        set_flags({k: v})

    def __contains__(self, k):
        return (k if k.startswith('FLAGS_') else 'FLAGS_' + k) in _REGISTRY

    def keys(self):
        return list(_REGISTRY.keys())

    def get(self, k, default=None):
        return self[k] if k in self else default

