"""Fused-epilogue GEMMs (EPI 2: bias+GELU writing h and gelu(h); EPI 3: dGELU reading h) vs the plain
bf16 GEMM of the same shape, interleaved rounds in one process (GPT-3 1.3B fc1 fwd / fc2 dgrad)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / n


def main():
    import paddle  # noqa: F401
    from paddle.ops import gemm, _native as N
    assert N._load() is not None
    M, K, F_, dev, bf = 16384, 2048, 8192, 'cuda', torch.bfloat16
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(bf)
    w1t = ((torch.rand(F_, K, device=dev) * 2 - 1) * 0.05).to(bf)  # K-major copy of W1 [K, F]
    b1 = torch.rand(F_, device=dev).to(bf)
    h = torch.empty(M, F_, device=dev, dtype=bf)
    dy = (torch.rand(M, K, device=dev) * 2 - 1).to(bf)
    w2 = ((torch.rand(F_, K, device=dev) * 2 - 1) * 0.05).to(bf)  # W2 [F, K] (in, out)
    fl = 2.0 * M * K * F_
    res = {k: [] for k in ('plain_fwd', 'epi2', 'plain_dgrad', 'epi3')}
    for _ in range(4):
        res['plain_fwd'].append(bench(lambda: gemm.mm(x, w1t.t(), bias=b1)))
        res['epi2'].append(bench(lambda: gemm.mm_epi(x, w1t.t(), 2, h, bias=b1)))
        res['plain_dgrad'].append(bench(lambda: gemm.mm(dy, w2.t())))
        res['epi3'].append(bench(lambda: gemm.mm_epi(dy, w2.t(), 3, h)))
    for k, v in res.items():
        t = min(v)
        print(f"{k:12s} {t*1e6:8.1f} us  {fl/t/1e12:6.0f} TF", flush=True)


if __name__ == '__main__':
    main()
