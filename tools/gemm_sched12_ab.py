"""A/B of the GEMM schedule (pa_gemm_set_variant: 0 = automatic 11 / 9, 12 = persistent with the
quarter-tile staged epilogue) on the GPT-3 1.3B GEMMs at M = 16384, interleaved rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def bench(fn, n=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    import paddle  # noqa: F401
    from paddle.ops import gemm, _native as N
    assert N._load() is not None
    M, dev, bf = 16384, 'cuda', torch.bfloat16
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(bf)  # noqa: E731
    cases = []
    for name, K, Nn in (('qkv fwd', 2048, 6144), ('out fwd', 2048, 2048), ('fc1 fwd', 2048, 8192),
                        ('fc2 fwd', 8192, 2048), ('lm fwd', 2048, 50304)):
        a, wt = r(M, K), r(Nn, K)
        cases.append((name, (lambda a=a, wt=wt: gemm.hip_mm(a, wt.t())), 2.0 * M * K * Nn))
    x, dy, gw = r(M, 2048), r(M, 8192), torch.zeros(2048, 8192, device=dev, dtype=bf)
    cases.append(('fc1 wgrad', lambda: gemm.hip_mm(x.t(), dy, out=gw, beta=1.0), 2.0 * M * 2048 * 8192))
    res = {}
    for rnd in range(3):
        for name, fn, fl in cases:
            for nt in (0, 1):
                N.lib.pa_gemm_set_variant(12 if nt else 0)
                res.setdefault((name, nt), []).append(bench(fn))
    N.lib.pa_gemm_set_variant(0)
    for name, fn, fl in cases:
        a_ = sorted(res[(name, 0)])[1]
        b_ = sorted(res[(name, 1)])[1]
        print(f"{name:14s} s11/9 {a_:8.1f} us ({fl / a_ / 1e6:5.0f} TF) | s12 {b_:8.1f} us ({fl / b_ / 1e6:5.0f} TF) | "
              f"{a_ / b_:5.3f}x", flush=True)


if __name__ == '__main__':
    main()
