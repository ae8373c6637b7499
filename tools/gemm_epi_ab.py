"""A/B of the schedule-11 epilogue (16-B permlane16-swap stores vs 8-B stores) on the GPT-3 1.3B
forward / dgrad shapes (M = 16384), interleaved rounds in one process, random operands."""
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
    M, dev, bf = 16384, 'cuda', torch.bfloat16
    shapes = [('qkv fwd', 2048, 6144), ('out fwd', 2048, 2048), ('fc1 fwd', 2048, 8192), ('fc2 fwd', 8192, 2048),
              ('fc2 dgrad', 2048, 8192), ('lm fwd', 2048, 50304)]
    for name, K, Nn in shapes + [('fc1 wgrad', 16384, -8192), ('out wgrad', 16384, -2048)]:
        if Nn < 0:  # weight gradient W[2048, N] += X^T @ dY: m-contiguous A (schedule 9), beta = 1
            Nn = -Nn
            xx = (torch.rand(K, 2048, device=dev) * 2 - 1).to(bf)
            dy = (torch.rand(K, Nn, device=dev) * 2 - 1).to(bf)
            gw = torch.zeros(2048, Nn, device=dev, dtype=bf)
            fl = 2.0 * K * 2048 * Nn
            ts, outs = {0: [], 1: []}, {}
            for rnd in range(3):
                for wide in (1, 0):
                    N.lib.pa_gemm8_set_wide_epi(wide)
                    ts[wide].append(bench(lambda: gemm.mm(xx.t(), dy, out=gw, beta=1.0)))
                    if rnd == 0:
                        outs[wide] = gemm.mm(xx.t(), dy, out=torch.zeros_like(gw), beta=1.0)
            N.lib.pa_gemm8_set_wide_epi(1)
            ref = xx.float().t() @ dy.float()
            e1 = (outs[1].float() - ref).abs().max().item()
            e0 = (outs[0].float() - ref).abs().max().item()
            t1, t0 = min(ts[1]), min(ts[0])
            print(f"{name:10s} K={K} N={Nn}: wide {t1*1e6:7.1f} us {fl/t1/1e12:5.0f} TF | narrow {t0*1e6:7.1f} us "
                  f"{fl/t0/1e12:5.0f} TF | {t0/t1:5.3f}x  err wide {e1:.3g} narrow {e0:.3g}", flush=True)
            continue
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(bf)
        w = (torch.rand(Nn, K, device=dev) * 2 - 1).to(bf)  # [N, K] k-contiguous B (kmajor copy / dgrad)
        bias = torch.rand(Nn, device=dev).to(bf)
        fl = 2.0 * M * K * Nn
        outs, ts = {}, {0: [], 1: []}
        for rnd in range(4):
            for wide in (1, 0):
                N.lib.pa_gemm8_set_wide_epi(wide)
                ts[wide].append(bench(lambda: gemm.mm(a, w.t(), bias=bias), 5 if Nn > 10000 else 10))
                if rnd == 0:
                    outs[wide] = gemm.mm(a, w.t(), bias=bias)
        N.lib.pa_gemm8_set_wide_epi(1)
        diff = (outs[1].float() - outs[0].float()).abs().max().item()
        ref = a.float() @ w.float().t() + bias.float()
        e1 = (outs[1].float() - ref).abs().max().item()
        e0 = (outs[0].float() - ref).abs().max().item()
        print(f"   err vs fp32: wide {e1:.3g} narrow {e0:.3g} (|ref| max {ref.abs().max().item():.3g})", flush=True)
        t1, t0 = min(ts[1]), min(ts[0])
        print(f"{name:10s} K={K} N={Nn}: wide {t1*1e6:7.1f} us {fl/t1/1e12:5.0f} TF | narrow {t0*1e6:7.1f} us "
              f"{fl/t0/1e12:5.0f} TF | {t0/t1:5.3f}x  maxdiff {diff:.3g}", flush=True)


if __name__ == '__main__':
    main()
