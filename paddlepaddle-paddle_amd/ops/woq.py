"""Weight-only int8 / int4 linear on the hand-written decode kernel (csrc/woq_gemm.hip): the
quantised weight is streamed once and dequantised in registers into MFMA fragments (W8A16 / W4A16),
for decode-shaped token counts (M <= 32).  Larger token counts dequantise once and run the
hand-written GEMM.  Reference: paddle/phi/kernels/gpu/weight_only_linear_kernel.cu."""
import torch

from . import _native as N

_DT = {torch.bfloat16: 1, torch.float16: 2}


def woq_ok(x2, wq, bits, group):
    if not x2.is_cuda or x2.dtype not in _DT or wq.dtype not in (torch.int8, torch.uint8) or x2.dim() != 2:
        return False
    if x2.stride(1) != 1 or wq.stride(1) != 1 or x2.data_ptr() % 16 or wq.data_ptr() % 16:
        return False
    if N._load() is None:
        return False
    M, K = x2.shape
    return bool(N.lib.pa_woq_ok(M, wq.shape[0], K, x2.stride(0), wq.stride(0), bits, group, _DT[x2.dtype]))


from .workspace import workspace as _workspace
_ws = _workspace('woq')


def woq_linear(x2, wq, scale, bits, group, bias=None):
    """x2 [M, K] bf16/fp16 @ dequant(wq [N, K(/2)])^T (+ bias) -> [M, N]."""
    M, K = x2.shape
    Nn = wq.shape[0]
    out = torch.empty(M, Nn, dtype=x2.dtype, device=x2.device)
    need = int(N.lib.pa_woq_ws_floats(M, Nn, K, bits))
    ws = _ws.get(need, torch.float32, x2.device, min_numel=1 << 20)
    sc = scale.float().contiguous()
    b = None if bias is None else bias.to(x2.dtype).contiguous()
    N.check(N.lib.pa_woq_gemm(N.ptr(x2), N.ptr(wq), N.ptr(sc), N.ptr(b), N.ptr(out), N.ptr(ws), M, Nn, K,
                              x2.stride(0), wq.stride(0), out.stride(0), bits, group, _DT[x2.dtype], N.stream()),
            'woq_gemm')
    return out
