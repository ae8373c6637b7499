"""int8 MFMA GEMM (csrc/gemm8x.hip pa_gemm8_i8, v_mfma_i32_16x16x64_i8) and per-token activation
quantisation (csrc/int8_quant.hip) — the kernels behind ``paddle.nn.quant.llm_int8_linear`` and the
int8 Linears of ``fused_multi_transformer`` (reference: paddle/phi/kernels/gpu/
llm_int8_linear_kernel.cu, python/paddle/nn/quant/quantized_linear.py:239)."""
import torch

from . import _native as N


def _lib():
    return N.lib if N.lib is not None else N._load()


def i8_mm_ok(a, w):
    """a: int8 [M, K] k-contiguous, w: int8 [N, K] k-contiguous (the quantised weight layout)."""
    if a.dtype != torch.int8 or w.dtype != torch.int8 or a.dim() != 2 or w.dim() != 2 or not a.is_cuda:
        return False
    if a.stride(1) != 1 or w.stride(1) != 1 or a.shape[1] != w.shape[1] or a.data_ptr() % 16 or w.data_ptr() % 16:
        return False
    return _lib() is not None and bool(N.lib.pa_gemm8_i8_ok(a.shape[0], w.shape[0], a.shape[1], a.stride(0),
                                                            w.stride(0), w.shape[0]))


def i8_mm(a, w, row_scale, col_scale, bias=None, out=None, beta=0.0, out_dtype=torch.bfloat16):
    """out[M, N] = (a @ w^T) * row_scale[m] * col_scale[n] (+ beta * out) (+ bias), int32 accumulation;
    row_scale fp32 [M] (per token), col_scale fp32 [N] (per output channel)."""
    M, K = a.shape
    Nn = w.shape[0]
    if out is None:
        out = torch.empty(M, Nn, dtype=out_dtype, device=a.device)
        beta = 0.0
    assert out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.shape == (M, Nn)
    rs = row_scale.float().contiguous()
    cs = col_scale.float().contiguous()
    b = None if bias is None else bias.to(torch.bfloat16).contiguous()
    N.check(N.lib.pa_gemm8_i8(N.ptr(a), N.ptr(w), N.ptr(out), N.ptr(b), N.ptr(rs), N.ptr(cs), M, Nn, K, a.stride(0),
                              w.stride(0), out.stride(0), float(beta), N.stream()), 'gemm8_i8')
    return out


def quant_rows(x, excl=None, rows=None):
    """Per-row absmax int8 quantisation of x [M, K] (bf16 / fp16 / fp32, k-contiguous): returns
    (q int8 [rows or M, K] — extra rows zero —, scale fp32 [rows or M]).  excl: uint8 [K], nonzero =
    column left out (quantised to 0, not counted in the absmax)."""
    M, K = x.shape
    R = rows or M
    q = torch.zeros(R, K, dtype=torch.int8, device=x.device) if R > M else \
        torch.empty(R, K, dtype=torch.int8, device=x.device)
    s = torch.ones(R, dtype=torch.float32, device=x.device)
    N.check(N.lib.pa_i8_quant_rows(N.ptr(x), M, K, x.stride(0), N.ptr(excl), N.ptr(q), K, N.ptr(s), N.dtcode(x.dtype),
                                   N.stream()), 'i8_quant_rows')
    return q, s


def quant_rows_ok(x):
    return (x.is_cuda and x.dim() == 2 and x.stride(1) == 1 and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.shape[1] % 8 == 0 and x.stride(0) % 8 == 0 and x.data_ptr() % 32 == 0 and _lib() is not None)
