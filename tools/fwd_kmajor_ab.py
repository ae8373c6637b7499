"""A/B of the Linear-forward weight layout on the hand-written GEMM (GPT-3 1.3B shapes):
(a) y = x @ W with W [in, out] read N-major straight from the parameter, vs
(b) W^T materialised by transpose2d each call, then y = x @ (W^T)^T (both operands K-major).
Run on the GPU: python tools/fwd_kmajor_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import paddle  # noqa: E402,F401
from paddle.ops import gemm  # noqa: E402


def timeit(fn, it=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it * 1e3


def main():
    dev = 'cuda'
    M = 16384
    for K, Nn, tag in ((2048, 6144, 'qkv'), (2048, 2048, 'out-proj'), (2048, 8192, 'fc1'), (8192, 2048, 'fc2')):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(K, Nn, device=dev) * 0.02).bfloat16()
        b = torch.zeros(Nn, device=dev).bfloat16()
        y = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
        ref = gemm.hip_mm(x, gemm.transpose2d(w).t())
        got = gemm.hip_mm(x, w)
        err = (got.float() - ref.float()).abs().max().item()
        fl = 2.0 * M * K * Nn
        ta = timeit(lambda: gemm.hip_mm(x, w, out=y))
        tt = timeit(lambda: gemm.transpose2d(w))
        tb = timeit(lambda: gemm.hip_mm(x, gemm.transpose2d(w).t(), out=y))
        line = (f"{tag:9s} M{M} K{K} N{Nn}: N-major W {ta:7.1f} us ({fl / ta / 1e6:6.0f} TF/s) | "
                f"transpose {tt:5.1f} us + K-major {tb - tt:7.1f} us = {tb:7.1f} us | max|diff| {err:.3g}")
        if tag == 'fc1':
            aux = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
            te_a = timeit(lambda: gemm.mm_epi(x, w, 2, aux, bias=b, out=y))
            te_b = timeit(lambda: gemm.mm_epi(x, gemm.transpose2d(w).t(), 2, aux, bias=b, out=y))
            line += f"\n{'':9s} epi2 (bias+GELU): N-major {te_a:7.1f} us | transpose+K-major {te_b:7.1f} us"
        print(line, flush=True)


if __name__ == '__main__':
    main()
