"""ERNIE-base Linear GEMMs (32768 tokens) fwd+dgrad+wgrad: library (torch.addmm autograd) vs the
hand-written kernels (ops.matmul.linear autograd, _LinearFn), bf16, interleaved rounds."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import paddle  # noqa: E402,F401
from paddle.ops import matmul as hm  # noqa: E402

T = 32768
shapes = [(768, 2304), (768, 768), (768, 3072), (3072, 768)]


def run(fn, x, w, b, g, it=20):
    for _ in range(3):
        fn(x, w, b).backward(g)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(it):
        fn(x, w, b).backward(g)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / it * 1e3


lib = lambda x, w, b: torch.addmm(b, x, w)  # noqa: E731
hip = lambda x, w, b: hm.linear(x, w, b)  # noqa: E731
for K, N in shapes:
    x = torch.randn(T, K, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(K, N, device='cuda', dtype=torch.bfloat16) * 0.02).requires_grad_()
    b = torch.zeros(N, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(T, N, device='cuda', dtype=torch.bfloat16)
    res = {'lib': [], 'hip': []}
    for _ in range(3):
        res['lib'].append(run(lib, x, w, b, g))
        res['hip'].append(run(hip, x, w, b, g))
    fl = 6 * T * K * N / 1e12
    print(f"[{T}x{K}]@[{K}x{N}] fwd+bwd  lib {min(res['lib']):.3f} ms ({fl / min(res['lib']) * 1e3:.0f} TF)  "
          f"hip {min(res['hip']):.3f} ms ({fl / min(res['hip']) * 1e3:.0f} TF)  hip/lib {min(res['lib']) / min(res['hip']):.2f}x",
          flush=True)
