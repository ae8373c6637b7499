"""Weight-only int8/int4 and LLM.int8 linear layers' functionals (reference:
python/paddle/nn/quant/quantized_linear.py).

Layout (ours, documented; the reference's is a CUTLASS-arch-specific interleave): a [k, n] float
weight quantises to int8 ``[n, k]`` (k contiguous) — int4 packs two signed nibbles per byte along
k into ``[n, k // 2]`` (per 8 k: byte b = k b low nibble, k 4 + b high nibble) — with symmetric absmax scales: per output channel
``[n]`` (group_size -1) or per k-group ``[k // group_size, n]``.  ``arch`` is accepted for API
compatibility (the MI355X path does not depend on it).  On the GPU, decode-shaped calls (<= 32 token
rows, bf16 / fp16) run the weight-only kernel csrc/woq_gemm.hip (quantised weight streamed once,
dequantised in registers into MFMA fragments); larger token counts dequantise once and run the
hand-written GEMM.
"""
import torch

from ...core.tensor import _wrap as _w, _unwrap as _u

_ALGOS = ('weight_only_int8', 'weight_only_int4', 'llm.int8')


def _check_group(group_size):
    if group_size not in (-1, 64, 128):
        raise ValueError(f"group_size must be -1, 64 or 128, got {group_size}")


def _qmax(algo):
    return 7.0 if algo == 'weight_only_int4' else 127.0


def weight_quantize(x, algo="weight_only_int8", arch=None, group_size=-1):
    """Quantise a [k, n] weight.  Returns (out, scale): out int8 [n, k] ([n, k // 2] packed for
    int4), scale float32 [n] (or [k // group_size, n])."""
    if algo not in _ALGOS:
        raise ValueError(f"algo must be one of {_ALGOS}, got {algo}")
    _check_group(group_size)
    w = _u(x).float()
    k, n = w.shape
    qm = _qmax(algo)
    if group_size == -1:
        scale = w.abs().amax(0).clamp_min(1e-12) / qm                       # [n]
        q = torch.round(w / scale).clamp(-qm, qm)
    else:
        if k % group_size:
            raise ValueError("k must be a multiple of group_size")
        wg = w.reshape(k // group_size, group_size, n)
        scale = wg.abs().amax(1).clamp_min(1e-12) / qm                      # [k/g, n]
        q = torch.round(wg / scale[:, None, :]).clamp(-qm, qm).reshape(k, n)
    q = q.to(torch.int8).t().contiguous()                                   # [n, k]
    if algo == 'weight_only_int4':
        if k % 8:
            raise ValueError("int4 packing needs k % 8 == 0")
        # per 8 consecutive k (one 32-bit word): byte b holds k 8w + b (low nibble) and 8w + 4 + b
        # (high nibble) — the decode kernel turns a word's low / high nibbles into two 4-element runs
        # of MFMA operand with one byte permute per pair (csrc/woq_gemm.hip frag_u4)
        q8 = q.to(torch.int16).reshape(n, k // 8, 2, 4) & 0xF
        q = (q8[:, :, 0] | (q8[:, :, 1] << 4)).reshape(n, k // 2).to(torch.uint8).view(torch.int8)  # [n, k/2]
        out = _w(q)
        out.__dict__['int4_layout'] = INT4_LAYOUT  # the packing travels with the tensor
        return out, _w(scale.float())
    return _w(q), _w(scale.float())


# int4 packing layouts: 1 = byte i holds k 2i (low nibble) and 2i + 1 (high) — the pre-round-5
# format; 2 = per 32-bit word w, byte b holds k 8w + b (low) and 8w + 4 + b (high) — the current one.
INT4_LAYOUT = 2


def convert_int4_layout(q, from_layout=1, to_layout=INT4_LAYOUT):
    """Re-pack an int4 weight ([n, k // 2] int8) between packing layouts (weights saved in the old
    pair layout decode to wrong values if fed to the current kernels unconverted)."""
    if from_layout == to_layout:
        return q
    t = _u(q).view(torch.uint8).to(torch.int16)
    n = t.shape[0]
    lo, hi = t & 0xF, (t >> 4) & 0xF
    if from_layout == 1:
        codes = torch.stack([lo, hi], -1).reshape(n, -1)                           # [n, k] in k order
    else:
        codes = torch.stack([lo.reshape(n, -1, 4), hi.reshape(n, -1, 4)], 2).reshape(n, -1)
    k = codes.shape[1]
    if to_layout == 1:
        c = codes.reshape(n, k // 2, 2)
        packed = c[..., 0] | (c[..., 1] << 4)
    else:
        if k % 8:
            raise ValueError("int4 layout 2 needs k % 8 == 0")
        c = codes.reshape(n, k // 8, 2, 4)
        packed = (c[:, :, 0] | (c[:, :, 1] << 4)).reshape(n, k // 2)
    out = _w(packed.to(torch.uint8).view(torch.int8).contiguous())
    out.__dict__['int4_layout'] = to_layout
    return out


def _unpack(q, algo):
    q = _u(q)
    if algo != 'weight_only_int4':
        return q.float()
    b = q.view(torch.uint8).to(torch.int16)
    lo, hi = b & 0xF, (b >> 4) & 0xF
    lo = torch.where(lo > 7, lo - 16, lo)
    hi = torch.where(hi > 7, hi - 16, hi)
    n = q.shape[0]
    return torch.stack([lo.reshape(n, -1, 4), hi.reshape(n, -1, 4)], 2).reshape(n, -1).float()  # [n, k]


def _dequant(q, scale, algo, group_size):
    v = _unpack(q, algo)                                                     # [n, k]
    s = _u(scale).float()
    if group_size == -1:
        return (v * s[:, None]).t()                                          # [k, n]
    n, k = v.shape
    return (v.reshape(n, k // group_size, group_size) * s.t()[:, :, None]).reshape(n, k).t()


def weight_dequantize(x, scale, algo="weight_only_int8", out_dtype='float16', group_size=-1):
    """Inverse of weight_quantize: the [k, n] weight in ``out_dtype``."""
    if algo not in _ALGOS:
        raise ValueError(f"algo must be one of {_ALGOS}, got {algo}")
    _check_group(group_size)
    from ...core.dtype import to_torch_dtype
    dt = to_torch_dtype(out_dtype)
    if dt not in (torch.float16, torch.bfloat16, torch.float32):
        raise ValueError("out_dtype must be float16 or bfloat16")
    return _w(_dequant(x, scale, algo, group_size).to(dt).contiguous())


def weight_only_linear(x, weight, bias=None, weight_scale=None, weight_dtype="int8", arch=None, group_size=-1):
    """y = x @ dequant(weight) (+ bias); weight/scale as produced by weight_quantize."""
    if weight_dtype not in ('int8', 'int4'):
        raise ValueError("weight_dtype must be 'int8' or 'int4'")
    _check_group(group_size)
    if weight_scale is None:
        raise ValueError("weight_only_linear needs weight_scale")
    t = _u(x)
    algo = 'weight_only_int4' if weight_dtype == 'int4' else 'weight_only_int8'
    if weight_dtype == 'int4' and getattr(weight, '__dict__', {}).get('int4_layout', INT4_LAYOUT) != INT4_LAYOUT:
        weight = convert_int4_layout(weight, weight.__dict__['int4_layout'])  # tagged old packing
    from ... import ops
    x2 = t.reshape(-1, t.shape[-1])
    wq = _u(weight)
    bits, grp = (4 if weight_dtype == 'int4' else 8), (0 if group_size == -1 else group_size)
    needs_grad = torch.is_grad_enabled() and (t.requires_grad or (bias is not None and _u(bias).requires_grad))
    if not needs_grad and ops.use_hip(x2) and ops.woq.woq_ok(x2.contiguous(), wq, bits, grp):
        # decode-shaped: stream the quantised weight once, dequantise in registers (csrc/woq_gemm.hip)
        y = ops.woq.woq_linear(x2.contiguous(), wq, _u(weight_scale), bits, grp,
                               None if bias is None else _u(bias))
        return _w(y.reshape(*t.shape[:-1], y.shape[-1]))
    w = _dequant(weight, weight_scale, algo, group_size).to(t.dtype)
    from ...tensor.linalg import matmul
    y = matmul(_w(t), _w(w.contiguous()))
    if bias is not None:
        y = _w(_u(y) + _u(bias).to(t.dtype))
    return y


# outlier-column capacity of the GPU path (a multiple of 64: the 16-bit outlier GEMM's K)
LLM_INT8_OUTLIER_CAP = 128
_OVERFLOW = {'flag': None, 'seen': False}


def llm_int8_linear(x, weight, bias=None, weight_scale=None, threshold=6.0):
    """LLM.int8 (reference quantized_linear.py:239 llm_int8_linear): input feature columns holding any
    |x| > threshold are multiplied in floating point with the dequantised weight rows; the rest are
    quantised per token (absmax, int8) and multiplied against the int8 weight, rescaled by both
    scales.

    On the GPU (bf16 / fp16 x, K % 128 == 0, N % 8 == 0) there is no host synchronisation: the
    outlier columns are compacted on the device into a fixed-capacity set (``LLM_INT8_OUTLIER_CAP``
    columns, outliers first by a stable device sort) whose 16-bit product runs on the hand-written
    GEMM with the bias, then the int8 MFMA GEMM (csrc/gemm8x.hip pa_gemm8_i8, int32 accumulation,
    per-token x per-channel dequant in its epilogue) accumulates onto it (beta = 1).  Every outlier
    column is excluded from the int8 row quantisation (row scales are never inflated by them).
    Should more columns than the capacity exceed the threshold, the surplus ones contribute nothing
    on that call; the overflow is detected on the device and read back without a sync (pinned
    flag, checked on the next call), which warns once and sends every later call of the process to
    the exact composite.  Elsewhere: the exact composite."""
    if weight_scale is None:
        raise ValueError("llm_int8_linear needs weight_scale")
    t = _u(x)
    lead = t.shape[:-1]
    qw_i8 = _u(weight)
    ws = _u(weight_scale)
    K = t.shape[-1]
    a16 = t.reshape(-1, K)
    from ... import ops
    if _OVERFLOW['flag'] is not None and bool(_OVERFLOW['flag'][0]) and not _OVERFLOW['seen']:
        import warnings
        _OVERFLOW['seen'] = True
        warnings.warn(f"llm_int8_linear: more than {LLM_INT8_OUTLIER_CAP} outlier columns above the threshold; "
                      "later calls use the exact composite path", RuntimeWarning)
    if (not _OVERFLOW['seen'] and a16.is_cuda and a16.dtype in (torch.bfloat16, torch.float16) and ops.use_hip(a16)
            and K % 128 == 0
            and qw_i8.dtype == torch.int8 and qw_i8.dim() == 2 and qw_i8.shape[1] == K and qw_i8.shape[0] % 8 == 0):
        y = _llm_int8_gpu(a16.contiguous(), qw_i8.contiguous(), ws, None if bias is None else _u(bias), threshold)
        if y is not None:
            return _w(y.to(t.dtype).reshape(*lead, -1))
    a = a16.float()
    qw = qw_i8.float()                                                       # [n, k] int8 values
    wsf = ws.float()                                                         # [n]
    outl = (a.abs() > threshold).any(0)                                      # [k]
    a_in = a.masked_fill(outl[None, :], 0.0)
    sx = a_in.abs().amax(1, keepdim=True).clamp_min(1e-12) / 127.0           # [m, 1]
    qa = torch.round(a_in / sx).clamp(-127, 127)
    y = (qa @ qw.t()) * sx * wsf[None, :]
    y = y + (a * outl[None, :].float()) @ (qw * wsf[:, None]).t()            # outlier columns, fp32
    if bias is not None:
        y = y + _u(bias).float()
    return _w(y.to(t.dtype).reshape(*lead, -1))


def _llm_int8_gpu(a, qw, ws, bias, threshold):
    from ...ops import int8 as I8, matmul as hm
    M, K = a.shape
    Nn = qw.shape[0]
    M8 = -(-M // 8) * 8
    if not I8.quant_rows_ok(a):
        return None
    cap = min(K, LLM_INT8_OUTLIER_CAP)
    outl = (a.abs() > threshold).any(0)                                      # [K] bool, device
    order = torch.argsort((~outl).to(torch.int8), stable=True)               # outlier columns first
    idx = order[:cap]
    sel = outl.index_select(0, idx)                                          # which of them are outliers
    excl = outl.to(torch.uint8)                                              # every outlier column
    qa, sx = I8.quant_rows(a, excl, rows=M8)                                 # int8 [M8, K], fp32 [M8]
    # capacity overflow: a device flag copied to pinned host memory without a sync (checked on the
    # next call, llm_int8_linear)
    if _OVERFLOW['flag'] is None:
        _OVERFLOW['flag'] = torch.zeros(1, dtype=torch.bool, pin_memory=True)
    _OVERFLOW['flag'].copy_((outl.sum() > cap).reshape(1), non_blocking=True)
    # 16-bit outlier product (+ bias) first: [M, cap] @ [cap, N]
    a_o = a.index_select(1, idx) * sel.to(a.dtype)
    w_o = (qw.index_select(1, idx).float() * ws.float()[:, None]).to(a.dtype).t().contiguous()
    a_o8 = a_o if M8 == M else torch.cat([a_o, a_o.new_zeros(M8 - M, cap)])
    b = None if bias is None else bias.to(a.dtype)
    out = hm.linear(a_o8, w_o, b)
    if out.dtype != torch.bfloat16:
        out = out.to(torch.bfloat16)
    if not I8.i8_mm_ok(qa, qw):
        return None
    out = I8.i8_mm(qa, qw, sx, ws, out=out.contiguous(), beta=1.0)
    return out[:M]


def apply_per_channel_scale(x, scales):
    """x * scales along the last (channel) dim (smooth-quant pre-scaling)."""
    t = _u(x)
    return _w(t * _u(scales).to(t.dtype))
