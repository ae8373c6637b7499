"""fp8 weight-gradient GEMMs of the ERNIE-base step (in x out features over 32768 tokens) under
split-K block budgets 256 / 384 / 512 (ops/gemm.py FP8_SPLITK_MAX_BLOCKS), device time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def t_us(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it * 1e3


def main():
    import paddle  # noqa: F401
    from paddle.ops import gemm as G, fp8 as F8, _native
    assert _native._load() is not None
    K = 32768
    sa = torch.ones(1, device='cuda')
    for M, N in ((768, 2304), (768, 768), (768, 3072), (3072, 768)):
        a = torch.randn(M, K, device='cuda').to(F8.E4M3)
        b = torch.randn(N, K, device='cuda').to(F8.E5M2)
        out = torch.empty(M, N, device='cuda', dtype=torch.bfloat16)
        res = []
        for cap in (256, 384):
            G.FP8_SPLITK_MAX_BLOCKS[0] = cap
            us = t_us(lambda: G.hip_fp8_mm(a, b, scale_a=sa, scale_b=sa, out=out, beta=1.0))
            res.append(f"cap {cap}: s={G._fp8_splitk(M, N, K):2d} {us:6.1f} us")
        print(f"[{M:5d} x {N:5d}] " + " | ".join(res), flush=True)


if __name__ == '__main__':
    main()
