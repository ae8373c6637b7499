"""Weight-only int8/int4 and LLM.int8 linear layers' functionals (reference:
python/paddle/nn/quant/quantized_linear.py).

Layout (ours, documented; the reference's is a CUTLASS-arch-specific interleave): a [k, n] float
weight quantises to int8 ``[n, k]`` (k contiguous) — int4 packs two signed nibbles per byte along
k into ``[n, k // 2]`` (low nibble = even k) — with symmetric absmax scales: per output channel
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
        if k % 2:
            raise ValueError("int4 packing needs an even k")
        lo = q[:, 0::2].to(torch.int16) & 0xF
        hi = q[:, 1::2].to(torch.int16) & 0xF
        q = (lo | (hi << 4)).to(torch.uint8).view(torch.int8)               # [n, k/2]
    return _w(q), _w(scale.float())


def _unpack(q, algo):
    q = _u(q)
    if algo != 'weight_only_int4':
        return q.float()
    b = q.view(torch.uint8).to(torch.int16)
    lo, hi = b & 0xF, (b >> 4) & 0xF
    lo = torch.where(lo > 7, lo - 16, lo)
    hi = torch.where(hi > 7, hi - 16, hi)
    return torch.stack([lo, hi], -1).reshape(q.shape[0], -1).float()        # [n, k]


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


def llm_int8_linear(x, weight, bias=None, weight_scale=None, threshold=6.0):
    """LLM.int8 (reference quantized_linear.py llm_int8_linear): input feature columns holding any
    |x| > threshold are multiplied in floating point with the dequantised weight rows; the rest are
    quantised per token (absmax, int8) and multiplied against the int8 weight, rescaled by both
    scales."""
    if weight_scale is None:
        raise ValueError("llm_int8_linear needs weight_scale")
    t = _u(x)
    lead = t.shape[:-1]
    a = t.reshape(-1, t.shape[-1]).float()
    qw = _u(weight).float()                                                  # [n, k] int8 values
    ws = _u(weight_scale).float()                                            # [n]
    outl = (a.abs() > threshold).any(0)                                      # [k]
    a_in = a.masked_fill(outl[None, :], 0.0)
    sx = a_in.abs().amax(1, keepdim=True).clamp_min(1e-12) / 127.0           # [m, 1]
    qa = torch.round(a_in / sx).clamp(-127, 127)
    y = (qa @ qw.t()) * sx * ws[None, :]
    if bool(outl.any()):
        y = y + a[:, outl] @ (qw[:, outl] * ws[:, None]).t()
    if bias is not None:
        y = y + _u(bias).float()
    return _w(y.to(t.dtype).reshape(*lead, -1))


def apply_per_channel_scale(x, scales):
    """x * scales along the last (channel) dim (smooth-quant pre-scaling)."""
    t = _u(x)
    return _w(t * _u(scales).to(t.dtype))
