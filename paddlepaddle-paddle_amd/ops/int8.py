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
    row_scale fp32 [M] (per token; None = 1), col_scale fp32 [N] (per output channel)."""
    M, K = a.shape
    Nn = w.shape[0]
    if out is None:
        out = torch.empty(M, Nn, dtype=out_dtype, device=a.device)
        beta = 0.0
    assert out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.shape == (M, Nn)
    rs = None if row_scale is None else row_scale.float().contiguous()
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


def quant_static(x, mul, rows=None, out_dtype=torch.int8, round_type=1, max_bound=127.0, min_bound=-127.0):
    """q = clip(round(x * mul), min_bound, max_bound) of x [M, K] (csrc/int8_quant.hip
    pa_i8_quant_static; round_type 1 rounds half away from zero, 0 half to even) into int8 — or bf16
    holding the same integers — [rows or M, K], padding rows zero."""
    M, K = x.shape
    R = rows or M
    q = torch.empty(R, K, dtype=out_dtype, device=x.device)
    N.check(_lib().pa_i8_quant_static(N.ptr(x), M, R, K, x.stride(0), N.ptr(q), K, float(mul), float(min_bound),
                                     float(max_bound), int(round_type), N.dtcode(x.dtype),
                                     0 if out_dtype == torch.int8 else 1, N.stream()), 'i8_quant_static')
    return q


def _round_ref(v, round_type):
    return torch.round(v) if round_type == 0 else torch.sign(v) * torch.floor(v.abs() + 0.5)


def static_int8_linear(x, qw, out_scale, in_scale, bias=None, round_type=1, max_bound=127.0, min_bound=-127.0):
    """The int8 Linear of fused_multi_transformer_int8 (reference fused_multi_transformer_int8_op.cu:
    quantise -> int8 GEMM -> dequantise + bias): x [..., K] is quantised per tensor with the
    calibrated ``in_scale`` (q = clip(round(max_bound * in_scale * x))), multiplied by the int8
    weight ``qw`` [N, K] in int32 and dequantised per output channel by ``out_scale`` [N]
    (y = acc * out_scale[n] + bias[n]).

    GPU: decode-shaped token counts (M <= 32) quantise into bf16 integers and stream the int8 weight
    once through the W8A16 decode kernel (csrc/woq_gemm.hip; integer products, fp32 sums; quantising
    inside that kernel's loads measured slower: every column block redoes it on its critical path); larger
    ones quantise into int8 rows (padded to 8) for the v_mfma_i32_16x16x64_i8 GEMM
    (csrc/gemm8x.hip pa_gemm8_i8) with the dequant scale and bias in its epilogue.  Output bf16 on
    the GPU (the model's activation dtype), x.dtype on the CPU composite."""
    from . import woq
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    M, Nn = x2.shape[0], qw.shape[0]
    mul = float(max_bound) * float(in_scale)
    osc = out_scale.to(device=x.device, dtype=torch.float32).reshape(-1)
    if x2.is_cuda and qw.dtype == torch.int8 and _lib() is not None and K % 8 == 0:
        x2 = x2.contiguous()
        if M <= 32:
            qb = quant_static(x2, mul, out_dtype=torch.bfloat16, round_type=round_type, max_bound=max_bound,
                              min_bound=min_bound)
            if woq.woq_ok(qb, qw, 8, 0):
                y = woq.woq_linear(qb, qw, osc, 8, 0, None if bias is None else bias.reshape(-1))
                return y.reshape(*x.shape[:-1], Nn)
        M8 = -(-M // 8) * 8
        qa = quant_static(x2, mul, rows=M8, round_type=round_type, max_bound=max_bound, min_bound=min_bound)
        if i8_mm_ok(qa, qw):
            y = i8_mm(qa, qw, None, osc, bias=None if bias is None else bias.reshape(-1))
            return y[:M].reshape(*x.shape[:-1], Nn)
    q = _round_ref(x2.float() * mul, round_type).clamp_(min_bound, max_bound)
    y = (q.double() @ qw.to(x.device).double().t()).float() * osc
    if bias is not None:
        y = y + bias.to(x.device).float().reshape(1, -1)
    return y.to(x.dtype if x.is_floating_point() else torch.float32).reshape(*x.shape[:-1], Nn)


# ----------------------------------------------------------------------------- static int8 programs
def quantize_static(x, scale, bits=8):
    """int8 q = clamp(round(x / step)) with a per-tensor (activation) step = scale / qmax."""
    qmax = float(2 ** (bits - 1) - 1)
    s = scale.to(x.device) if isinstance(scale, torch.Tensor) else torch.tensor(float(scale), device=x.device)
    step = s.float().reshape(()) / qmax
    return torch.round(x.float() / step).clamp_(-qmax, qmax).to(torch.int8)


def quant_linear(x, qw, w_scale, act_scale, bias=None, bits=8, weight_bits=8):
    """A frozen quantised Linear (paddle.static.quantization): y = dequant(quant(x)) @ dequant(qw)^T
    (+ bias) with x quantised per tensor by the calibrated ``act_scale`` (abs-max threshold) and the
    int8 weight ``qw`` [N, K] (k-contiguous) by per-output-channel ``w_scale`` [N] thresholds.
    On the GPU: the int8 MFMA GEMM (pa_gemm8_i8) with the two dequant steps in its epilogue."""
    qmax_a = float(2 ** (bits - 1) - 1)
    qmax_w = float(2 ** (weight_bits - 1) - 1)
    K = x.shape[-1]
    x2 = x.reshape(-1, K)
    M, Nn = x2.shape[0], qw.shape[0]
    ws = w_scale.to(device=x.device, dtype=torch.float32).reshape(-1) / qmax_w   # per-channel dequant step
    a_step = (act_scale.to(device=x.device, dtype=torch.float32) if isinstance(act_scale, torch.Tensor) else
              torch.tensor(float(act_scale), device=x.device)).reshape(()) / qmax_a
    if (x2.is_cuda and bits == 8 and weight_bits == 8 and K % 128 == 0 and Nn % 8 == 0 and qw.dtype == torch.int8
            and _lib() is not None):
        M8 = -(-M // 8) * 8
        qa = quantize_static(x2, act_scale, bits)
        if M8 != M:
            qa = torch.cat([qa, qa.new_zeros(M8 - M, K)])
        if i8_mm_ok(qa, qw.contiguous()):
            y = i8_mm(qa, qw.contiguous(), a_step.expand(M8).contiguous(), ws,
                      bias=None if bias is None else bias.reshape(-1))
            return y[:M].to(x.dtype if x.is_floating_point() else torch.bfloat16).reshape(*x.shape[:-1], Nn)
    xq = quantize_static(x2, act_scale, bits).float() * a_step
    y = xq @ (qw.to(x.device).float() * ws[:, None]).t()
    if bias is not None:
        y = y + bias.to(x.device).float()
    return y.to(x.dtype).reshape(*x.shape[:-1], Nn)


class _FakeQuant(torch.autograd.Function):
    """quant -> dequant with a straight-through gradient (inside the clip range)."""

    @staticmethod
    def forward(ctx, x, step, qmax):
        q = torch.round(x / step).clamp(-qmax, qmax)
        ctx.save_for_backward(x, step)
        ctx.qmax = qmax
        return q * step

    @staticmethod
    def backward(ctx, g):
        x, step = ctx.saved_tensors
        keep = (x.abs() <= step * ctx.qmax).to(g.dtype)
        return g * keep, None, None


def fake_quant_dequant(x, scale, bits=8, axis=None):
    """Quantise-dequantise x with abs-max threshold ``scale`` (per tensor, or per channel along
    ``axis``), straight-through gradient.  The QAT node of QuantizationTransformPass."""
    qmax = float(2 ** (bits - 1) - 1)
    s = scale.to(x.dtype) if isinstance(scale, torch.Tensor) else torch.tensor(float(scale), dtype=x.dtype,
                                                                              device=x.device)
    if axis is not None and s.dim() == 1:
        shape = [1] * x.dim()
        shape[axis] = -1
        s = s.reshape(shape)
    step = torch.clamp(s / qmax, min=1e-12)
    return _FakeQuant.apply(x, step, qmax)


def moving_average_abs_max(x, state, accum, moving_rate, training):
    """Activation fake quant of QAT (reference fake_quantize_dequantize_moving_average_abs_max):
    in training the threshold is the moving average accum / state of the batch abs-max, updated in
    place on the device; returns quant-dequant(x)."""
    if training:
        with torch.no_grad():
            cur = x.detach().abs().amax().float()
            state.mul_(moving_rate).add_(1.0)
            accum.mul_(moving_rate).add_(cur)
    scale = (accum / state.clamp(min=1e-12)).to(x.dtype)
    return fake_quant_dequant(x, scale)
