"""Decode-shaped GEMMs (M = batch of new tokens, Llama-2-13B layer weights): the path
fused_multi_transformer takes (ops.gemm.mm) vs the library (torch.matmul) vs the weight-streaming
bound (weight bytes / 6 TB/s)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddle  # noqa: E402,F401
from paddle.ops import gemm  # noqa: E402


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    E, F_ = 5120, 13824
    shapes = [('qkv', E, 3 * E), ('out', E, E), ('ffn1 (swiglu)', E, 2 * F_), ('ffn2', F_, E)]
    for M in (1, 8, 16, 32, 64):
        for name, K, N in shapes:
            x = torch.randn(M, K, device='cuda').to(torch.bfloat16)
            w = (torch.randn(K, N, device='cuda') * 0.02).to(torch.bfloat16)
            bound = K * N * 2 / 6e12 * 1e6
            t_mm = timeit(lambda: gemm.mm(x, w))
            t_lib = timeit(lambda: torch.matmul(x, w))
            y0, y1 = gemm.mm(x, w).float(), (x.float() @ w.float())
            err = (y0 - y1).abs().max().item()
            print(f"M {M:3d} {name:14s} K {K:5d} N {N:5d}: ops.gemm.mm {t_mm:8.1f} us | torch.matmul {t_lib:8.1f} us"
                  f" | bound {bound:6.1f} us | max err {err:.3g}")


if __name__ == '__main__':
    main()
