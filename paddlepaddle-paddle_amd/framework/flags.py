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


# Framework switches (MI355X kernel routing and engine knobs), registered as ``FLAGS_pa_<name>``:
# settable by set_flags / the FLAGS_pa_<name> environment variable, and — for scripts of earlier
# rounds — by the legacy PADDLE_AMD_<NAME> variable.  Most are read once at import by the module
# they configure (kernel routing is fixed per process).  name: (default, doc)
PA_FLAGS = {
    'disable_hip_kernels': (False, 'route every op to the ATen composite (A/B against the HIP kernels)'),
    'hip_gemm': (True, 'hand-written MFMA GEMM (csrc/gemm8.hip) for Linear / matmul'),
    'hip_matmul': (True, 'paddle.matmul / bmm / einsum on the hand-written GEMM when the operands fit'),
    'skinny_gemm': (True, 'decode-shaped GEMMs (M <= 64) on csrc/skinny_gemm.hip'),
    'gemm_autotune': (True, 'per-shape hand-written-vs-library choice for plain GEMMs (single rank)'),
    'gemm_tuning': (True, 'apply the measured per-shape GEMM schedule table (ops/gemm_tuning.py)'),
    'kmajor_fwd': (True, 'transient K-major weight copy for the Linear forward (>= 4096 rows)'),
    'fp8_8phase': (True, '8-phase fp8 GEMM schedule (else the 2-stage kernel)'),
    'wgrad_overlap': (False, 'weight-gradient GEMM on a side stream beside the data-gradient GEMM'),
    'group_wgrad': (True, 'group weight-gradient GEMMs whose tile counts fill one round of the chip'),
    'defer_fc2_bias': (True, 'GPT: fc2 bias gradient from the fused dgrad epilogue column sums'),
    'gemm_staged': ('', 'GEMM epilogue staging level override (0/1/2; empty: built-in default)'),
    'gemm_staged9': ('', 'weight-gradient epilogue staging override (empty: default)'),
    'conv_staged': ('', 'conv output staging override (empty: default)'),
    'fa_ds_bwd': ('', 'flash-attention backward form: 1 materialised dS, 0 recompute (empty: by shape)'),
    'fa_ds_ws_mb': (8192, 'flash-attention dS workspace cap (MiB)'),
    'hip_conv': (True, 'implicit-GEMM MFMA convolutions (csrc/conv.hip)'),
    'hip_conv_bwd': (True, 'data / filter gradients of convolutions on the HIP kernels'),
    'hip_conv_wgrad': (True, 'filter gradient on the HIP kernel'),
    'conv_bn_stats': (True, 'batch-norm statistics in the conv epilogue'),
    'conv1x1_gemm': (True, '1x1 stride-1 convolutions on the GEMM'),
    'conv_stem': (True, 'few-channel stem convolution kernel (csrc/conv_stem.hip)'),
    'hip_dwconv': (True, 'depthwise convolutions on csrc/dwconv.hip'),
    'hip_gconv': (True, 'grouped convolutions on csrc/gconv.hip'),
    'force_collectives': (False, 'run the real collectives at world size 1 (1-rank RCCL rehearsal)'),
    'sharding_alias': (True, 'world-1 sharding units alias the optimizer arenas'),
    'dist_to_static': (True, 'dist.to_static records a static Program (else eager SPMD)'),
    'sot_frontend': ('opcode', "SOT front end: 'opcode' (this framework's translator) or 'dynamo'"),
    'sot': (True, 'to_static(full_graph=False) runs through the bytecode (SOT) translator (jit/opcode_translator.py)'),
    'pdmodel': (True, 'save_inference_model writes the reference ProgramDesc format when possible'),
    'pir': ('', 'jit.save writes the PIR json program (1 / 0; empty: FLAGS_enable_pir_api)'),
}


def _parse(default, s):
    if isinstance(default, bool):
        return s.lower() in ('1', 'true', 'yes', 'on')
    if isinstance(default, int):
        return int(s)
    if isinstance(default, float):
        return float(s)
    return s


for _n, (_d, _doc) in PA_FLAGS.items():
    _REGISTRY['FLAGS_pa_' + _n] = _d
    _legacy = 'PADDLE_AMD_' + _n.upper()
    if _legacy in os.environ and ('FLAGS_pa_' + _n) not in os.environ:
        try:
            _REGISTRY['FLAGS_pa_' + _n] = _parse(_d, os.environ[_legacy])
        except ValueError:
            pass

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
        _EXPLICIT.add(k)
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



_EXPLICIT = set()


def pa_flag(name):
    """Value of the framework switch FLAGS_pa_<name> (PA_FLAGS): a value given by set_flags wins,
    then the live environment (FLAGS_pa_<name>, then the legacy PADDLE_AMD_<NAME>), then the
    default — switches read at construction time follow environment changes made at run time."""
    key = 'FLAGS_pa_' + name
    if key not in _EXPLICIT:
        d = PA_FLAGS[name][0]
        for env in (key, 'PADDLE_AMD_' + name.upper()):
            if env in os.environ:
                try:
                    return _parse(d, os.environ[env])
                except ValueError:
                    break
    return _REGISTRY[key]
