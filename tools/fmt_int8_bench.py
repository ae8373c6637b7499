"""Per-Linear latency of the int8 fused_multi_transformer path (ops.int8.static_int8_linear:
static quantisation + int8 MFMA GEMM / W8A16 decode kernel) against the bf16 GEMM of the same
shape (ops.gemm.mm), device time under hipGraph replay, on 13B-class layer shapes, decode (M = 1, 16) and prefill (M = 2048, 8192)."""
import json
import sys

import torch

sys.path.insert(0, '.')
import paddle  # noqa: E402,F401
from paddle import ops  # noqa: E402


def t_ms(fn, it=20, reps=5):
    """Device time per call: ``it`` calls captured in one hipGraph and replayed (decode runs
    captured — DecodeStepGraph — so host dispatch is not part of the per-Linear cost)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(it):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (it * reps)


def main():
    dev = 'cuda'
    shapes = {'qkv': (15360, 5120), 'out': (5120, 5120), 'ffn1': (27648, 5120), 'ffn2': (5120, 13824)}
    rows = []
    for M in (1, 16, 2048, 8192):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            wq = torch.randint(-127, 128, (N, K), device=dev, dtype=torch.int8)
            wb = torch.randn(K, N, device=dev, dtype=torch.bfloat16) * 0.02
            osc = torch.full((N,), 1e-4, device=dev)
            b = torch.randn(N, device=dev, dtype=torch.bfloat16)
            ti = t_ms(lambda: ops.int8.static_int8_linear(x, wq, osc, 0.3, b))
            tb = t_ms(lambda: ops.gemm.mm(x, wb, bias=b))
            fl = 2.0 * M * N * K
            rows.append(dict(M=M, layer=name, N=N, K=K, int8_us=round(ti * 1e3, 1), bf16_us=round(tb * 1e3, 1),
                             speedup=round(tb / ti, 3), int8_tops=round(fl / ti / 1e9, 1),
                             int8_weight_TBps=round(N * K / ti / 1e9, 2)))
            print(json.dumps(rows[-1]), flush=True)


if __name__ == '__main__':
    main()
