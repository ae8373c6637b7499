"""ctypes binding of ``_lib/libpaddle_amd_kernels.so`` (the hand-written HIP kernel library).

Every launcher takes raw device pointers and the caller's current HIP stream, so the
kernels interleave correctly with the storage layer's own work and can be captured into
hipGraphs.  A failed launch raises immediately (the hipError_t is checked per call).
"""
from ..framework.flags import pa_flag  # noqa: E402
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# PADDLE_AMD_KERNEL_LIB: another build of the kernel library (same-box A/B of two kernel versions)
LIB_PATH = os.environ.get('PADDLE_AMD_KERNEL_LIB') or os.path.join(_HERE, '_lib', 'libpaddle_amd_kernels.so')

lib = None
load_error = None

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
F = ctypes.c_float
U32 = ctypes.c_uint32
LLP = ctypes.POINTER(ctypes.c_longlong)

_SIGS = {
    'pa_layernorm_fwd': [P, P, P, P, P, P, P, P, I, I, F, I, I, P],
    'pa_rmsnorm_fwd': [P, P, P, P, P, P, I, I, F, I, I, P],
    'pa_layernorm_bwd': [P, P, P, P, P, P, P, P, P, P, I, I, I, I, P],
    'pa_rmsnorm_bwd': [P, P, P, P, P, P, P, P, I, I, I, I, P],
    'pa_norm_bwd_nparts': [I],
    'pa_dropout_add_norm_fwd': [P, P, P, P, P, P, P, P, P, I, I, F, I, F, U32, U32, I, I, P],
    'pa_dropout_add_norm_bwd': [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, F, U32, U32, I, I, P],
    'pa_colsum_nparts': [I, I, I],
    'pa_bias_act_bwd_dbias': [I, P, P, P, P, P, P, I, I, I, I, I, P],
    'pa_colsum': [P, P, P, I, I, I, I, I, P],
    'pa_transpose2d': [P, P, I, I, I, P],
    'pa_maxpool2d_nhwc_fwd': [P, P, P] + [I] * 13 + [P],
    'pa_dwconv_ok': [I] * 15,
    'pa_conv_stem_ok': [I] * 6,
    'pa_conv_stem_kp': [I, I, I],
    'pa_conv_stem_rk': [I, I],
    'pa_conv_stem_fwd': [P] * 5 + [I] * 14 + [P],
    'pa_conv_stem_stat_rows': [I],
    'pa_conv2d_fwd_pad_taps': [I, I, I],
    'pa_conv2d_fwd_cpad': [I],
    'pa_gconv_ok': [I] * 17,
    'pa_gconv_fwd': [P] * 4 + [I] * 17 + [P],
    'pa_gconv_dgrad': [P] * 3 + [I] * 17 + [P],
    'pa_gconv_wgrad_splits': [I] * 8,
    'pa_gconv_wgrad': [P] * 4 + [I] * 19 + [P],
    'pa_dwconv_fwd': [P, P, P, P] + [I] * 15 + [P],
    'pa_dwconv_dgrad': [P, P, P] + [I] * 15 + [P],
    'pa_dwconv_wgrad_splits': [I] * 6,
    'pa_dwconv_wgrad': [P, P, P, P] + [I] * 17 + [P],
    'pa_maxpool2d_nhwc_bwd': [P, P, P] + [I] * 13 + [P],
    'pa_bn_ws_floats': [I, I, I],
    'pa_bn_fwd': [P, P, P, P, P, P, P, P, P, P, I, I, F, F, I, I, I, I, P],
    'pa_bn_fwd_parts': [P, P, P, P, P, P, P, P, P, P, I, I, P, I, I, F, F, I, I, I, P],
    'pa_bn_bwd': [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, P],
    'pa_softmax_fwd': [P, P, I, I, I, I, P],
    'pa_softmax_bwd': [P, P, P, I, I, I, P],
    'pa_xent_fwd': [P, P, P, P, I, I, LL, I, P],
    'pa_xent_bwd': [P, P, P, P, I, P, I, I, LL, I, P],
    'pa_bias_act': [I, I, P, P, P, P, LL, I, I, P],
    'pa_swiglu_fwd': [P, P, P, LL, I, I, I, P],
    'pa_swiglu_bwd': [P, P, P, P, P, LL, I, I, I, P],
    'pa_dropout_add_fwd': [P, P, P, LL, F, U32, U32, I, P],
    'pa_dropout_bwd': [P, P, LL, F, U32, U32, I, P],
    'pa_embedding_fwd': [P, P, P, I, I, LL, I, P],
    'pa_embedding_bwd': [P, P, P, P, I, I, LL, I, I, P],
    'pa_embedding_bwd_pad': [P, P, P, P, I, I, LL, I, LL, I, P],
    'pa_rope': [P, P, P, P, P, I, I, I, I, I, F, I, P],
    'pa_rope_rows': [P, LL, P, LL, P, P, P, I, I, I, I, I, F, I, P],
    'pa_adamw': [P, P, P, P, P, LL, P, F, F, F, F, F, F, F, P, P, I, I, P],
    'pa_sumsq': [P, LL, P, I, P],
    'pa_momentum': [P, P, P, P, LL, P, F, F, F, F, I, P, I, I, P],
    'pa_sumsq_parts': [],
    'pa_gemm_set_variant': [I],
    'pa_adamw_tune': [I, I],
    'pa_act_fwd_tune': [I, I],
    'pa_act_cs_tune': [I],
    'pa_flash_set_bwd_variant': [I],
    'pa_flash_set_pair_group': [I],
    'pa_flash_set_fwd_pipe': [I],
    'pa_flash_set_fwd_sp': [I],
    'pa_gemm_fp8_ok': [I, I, I, LL, LL, LL],
    'pa_fp8_cast_transpose': [P, I, I, LL, P, P, P, I, I, P, I, F, P],
    'pa_fp8_cast_transpose_cs': [P, I, I, LL, P, P, P, I, I, P, I, F, P, P],
    'pa_fp8_amax': [P, I, I, LL, P, P],
    'pa_fp8_cast_transpose_multi': [P, I, I, I, P],
    'pa_norm_set_bwd_wave': [I],
    'pa_fp8_set_cast_full': [I],
    'pa_woq_tune': [I, I],
    'pa_woq_set_ct': [I],
    'pa_woq_set_fused_finish': [I],
    'pa_gemm_fp8': [P, P, P, P, P, P, I, I, I, LL, LL, LL, F, F, I, I, P],
    'pa_gemm8_fp8_ok': [I, I, I, LL, LL, LL],
    'pa_gemm8_fp8': [P, P, P, P, P, P, I, I, I, LL, LL, LL, F, F, I, I, P],
    'pa_gemm8_fp8_epi': [P, P, P, P, P, P, P, I, I, I, LL, LL, LL, F, I, I, I, P],
    'pa_gemm8_fp8_epi_q': [P, P, P, P, P, P, P, P, P, P, I, I, I, LL, LL, F, I, I, P],
    'pa_fp8_scale_prep': [P, I, I, I, F, P, P, P],
    'pa_gemm8_i8_ok': [I, I, I, LL, LL, LL],
    'pa_gemm8_i8': [P, P, P, P, P, P, I, I, I, LL, LL, LL, F, P],
    'pa_i8_quant_rows': [P, I, I, LL, P, P, LL, P, I, P],
    'pa_i8_quant_static': [P, I, I, I, LL, P, LL, F, F, F, I, I, I, P],
    'pa_amp_check_unscale': [P, P, P, I, P, P, P],
    'pa_amp_update_scale': [P, P, P, P, I, I, F, F, F, P],
    'pa_gemm8_fp8_splitk': [P, P, P, P, P, P, P, I, I, I, LL, LL, LL, F, F, I, I, I, P],
    'pa_gemmx_ok': [I, I, I, LL, LL, LL, I, I, I],
    'pa_woq_ok': [I, I, I, LL, LL, I, I, I],
    'pa_woq_ws_floats': [I, I, I, I],
    'pa_woq_gemm': [P, P, P, P, P, P, I, I, I, LL, LL, LL, I, I, I, P],
    'pa_gemmx': [P, P, P, P, I, I, I, LL, LL, LL, I, I, I, LL, LL, LL, I, F, F, P],
    'pa_conv2d_fwd_ok': [I, I, I, I],
    'pa_conv2d_fwd': [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P],
    'pa_conv2d_fwd_stats': [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P],
    'pa_conv2d_fwd_stat_rows': [I],
    'pa_im2col_nhwc': [P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P],
    'pa_im2col_rows_ok': [I, I],
    'pa_norm_set_rng_gen': [P],
    'pa_skinny_ok': [I, I, I, LL, LL],
    'pa_skinny_ws_floats': [I, I, I],
    'pa_skinny_gemm': [P, P, P, P, P, I, I, I, LL, LL, LL, I, P],
    'pa_act_set_rng_gen': [P],
    'pa_flash_set_rng_gen': [P],
    'pa_flash_ds_set_rng_gen': [P],
    'pa_flash_ds_ld': [I],
    'pa_flash_ds_ws_elems': [I, I, I, I],
    'pa_flash_ds_set_pair_group': [I],
    'pa_flash_ds_set_dq_dma': [I],
    'pa_flash_bwd_ds': [P] * 11 + [I] * 6 + [LLP] * 8 + [F, I, I, P, P, I, P, LL, LL, LL, I, F, U32, U32, P, LL, LL, P,
                                                         P],
    'pa_conv2d_wgrad_ok': [I, I],
    'pa_conv2d_dgrad_classes': [P, P, P, I, I, I, I, I, I, I, I, I, I, P, P, P, P],
    'pa_conv2d_wgrad': [P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, I, P],
    'pa_conv2d_wgrad_splits': [I, I, I, I],
    'pa_conv2d_wgrad_set_bncap': [I],
    'pa_conv2d_wgrad_set_wm': [I],
    'pa_conv2d_set_wm': [I, I],
    'pa_conv2d_set_staged': [I],
    'pa_gemm_ok': [I, I, I, LL, LL, LL, I],
    'pa_gemm8_ok': [I, I, I, LL, LL, LL, I, I, I],
    'pa_gemm8_set_wide_epi': [I],
    'pa_gemm8_set_nt_store': [I],
    'pa_gemm8_set_epi_sched': [I],
    'pa_gemm8_diag': [P, P, P, P, P, I, I, I, I, P],
    'pa_gemm8_set_staged_epi': [I],
    'pa_gemm8_set_staged9': [I],
    'pa_bn_tune': [I],
    'pa_bn_set_interleave': [I],
    'pa_conv_set_wgrad_direct': [I],
    'pa_act_cs_set_interleave': [I],
    'pa_colsum_finish_parts': [P, P, I, I, I, I, P],
    'pa_gemm8_bf16_epi': [P, P, P, P, P, I, I, I, LL, LL, LL, I, F, I, P],
    'pa_gemm8_bf16_act': [P, P, P, P, I, I, I, LL, LL, LL, I, F, I, P],
    'pa_gemm8_wgrad_grouped2': [P, P, P, I, I, LL, LL, LL, P, P, P, I, I, LL, LL, LL, I, F, F, P],
    'pa_gemm_bf16': [P, P, P, P, P, I, I, I, LL, LL, LL, I, I, F, F, I, P],
    'pa_flash_fwd_ex': [P, P, P, P, P, I, I, I, I, I, I, LLP, LLP, LLP, LLP, F, I, I, P, P, I, P, LL, LL, LL, I, F,
                        U32, U32, P, LL, LL, P, P],
    'pa_flash_bwd_ex': [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, LLP, LLP, LLP, LLP, LLP, LLP, LLP, LLP, F, I,
                        I, P, P, I, P, LL, LL, LL, I, F, U32, U32, P, LL, LL, P, P],
    'pa_decode_nsplit': [I, I, I],
    'pa_decode_ok': [I, I, I],
    'pa_decode_attn': [I, P, LL, P, P, P, P, I, I, LL, P, P, LL, P, LL, P, I, I, I, I, I, F, P],
    'pa_decode_attn_q8': [I, P, LL, P, P, P, P, I, I, LL, P, P, LL, P, LL, P, I, I, I, I, I, F, P, P, LL, P],
    'pa_kv_cache_write': [I, P, P, LL, P, P, P, P, P, I, I, LL, P, P, I, I, I, P],
    'pa_kv_cache_write_q8': [I, I, P, P, LL, P, P, P, I, I, LL, P, P, I, I, I, P, P, LL, I, F, F, P],
    'pa_flash_fwd': [P, P, P, P, P, I, I, I, I, I, I, LLP, LLP, LLP, LLP, F, I, I, P],
    'pa_flash_bwd': [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, LLP, LLP, LLP, LLP, LLP, LLP, LLP, LLP, F, I, I,
                     P],
}

_LL_RET = {'pa_bn_ws_floats', 'pa_skinny_ws_floats', 'pa_woq_ws_floats', 'pa_flash_ds_ws_elems'}
_VOID_RET = {'pa_adamw_tune', 'pa_act_fwd_tune', 'pa_act_cs_tune'}


def _load():
    global lib, load_error
    if lib is not None:
        return lib
    if not os.path.exists(LIB_PATH):
        load_error = f"{LIB_PATH} not built (run __graft_entry__.build() or python paddlepaddle-paddle_amd/_build.py)"
        return None
    try:
        l = ctypes.CDLL(LIB_PATH)
        for name, args in _SIGS.items():
            fn = getattr(l, name)
            fn.argtypes = args
            fn.restype = None if name in _VOID_RET else (ctypes.c_longlong if name in _LL_RET else ctypes.c_int)
        lib = l
        st = (pa_flag('gemm_staged') or None)  # A/B: LDS-staged GEMM epilogue level (0/1/2)
        if st is not None:
            l.pa_gemm8_set_staged_epi(int(st))
        cst = (pa_flag('conv_staged') or None)  # A/B: staged conv output stores
        if cst is not None:
            l.pa_conv2d_set_staged(int(cst))
        st9 = (pa_flag('gemm_staged9') or None)  # A/B: staged weight-gradient epilogue
        if st9 is not None:
            l.pa_gemm8_set_staged9(int(st9))
    except OSError as e:  # pragma: no cover
        load_error = str(e)
    return lib


def check(err, name):
    if err != 0:
        raise RuntimeError(f"HIP kernel launch {name} failed with hipError_t={err}")


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def ptr(t):
    """Device pointer of a GPU tensor for a kernel argument.  Anything else (a CPU tensor, or a
    meta tensor recorded into a static Program) raises here instead of reaching a kernel."""
    if t is None:
        return None
    if t.device.type != 'cuda':
        raise RuntimeError(f"HIP kernel operand on {t.device} (expected a GPU tensor)")
    return ctypes.c_void_p(t.data_ptr())


def dtcode(dt):
    if dt == torch.float32:
        return 0
    if dt == torch.bfloat16:
        return 1
    if dt == torch.float16:
        return 2
    raise TypeError(f"unsupported dtype for HIP kernel: {dt}")


def strides3(t):
    """(batch, seq, head) element strides of a [B, S, H, D] tensor with unit D stride."""
    s = t.stride()
    arr = (ctypes.c_longlong * 3)(s[0], s[1], s[2])
    return arr
