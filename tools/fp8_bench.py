"""FP8 training Linear vs the bf16 Linear on the GPT-3 1.3B step's shapes (M = 16 x 1024 tokens).

Per shape: forward + backward (dgrad + wgrad) of one Linear,
  bf16: y = x @ W on the hand-written bf16 GEMMs (ops.gemm.hip_mm, the training step's path)
  fp8 : ops.fp8._FP8Linear (HIP cast+transpose with delayed scaling, three fp8 MFMA GEMMs)
plus the bare fp8 GEMM against torch._scaled_mm and the cast kernel's bandwidth.  Random operands.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=10):
    for _ in range(3):
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
    from paddle.ops import gemm, fp8 as F8, _native
    assert _native._load() is not None, _native.load_error
    M, dev, bf = 16 * 1024, 'cuda', torch.bfloat16
    for name, K, N in [('qkv', 2048, 6144), ('out', 2048, 2048), ('fc1', 2048, 8192), ('fc2', 8192, 2048)]:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(bf).requires_grad_()
        w = ((torch.rand(K, N, device=dev) * 2 - 1) * 0.02).to(bf).requires_grad_()
        g = (torch.rand(M, N, device=dev) * 2 - 1).to(bf)
        fl = 3 * 2.0 * M * K * N

        def bf16_step():
            y = gemm.mm(x.detach(), w.detach())
            gemm.mm(g, w.detach().t())          # dgrad
            gemm.mm(x.detach().t(), g)          # wgrad
            return y

        st = F8.FP8State(F8.DelayedScaling(), dev)

        def fp8_step():
            y = F8._FP8Linear.apply(x, w, None, st)
            y.backward(g)
            x.grad = w.grad = None
            return y

        tb, tf = bench(bf16_step), bench(fp8_step)
        print(f"linear fwd+bwd {name} K={K} N={N}: bf16 {tb*1e6:8.1f} us {fl/tb/1e12:6.0f} TF | "
              f"fp8 {tf*1e6:8.1f} us {fl/tf/1e12:6.0f} TF  speedup {tb/tf:4.2f}x", flush=True)
        a = (torch.rand(M, K, device=dev) * 2 - 1).to(F8.E4M3)
        bt = (torch.rand(N, K, device=dev) * 2 - 1).to(F8.E4M3)
        one = torch.ones((), device=dev)
        f1 = 2.0 * M * K * N
        tl = bench(lambda: torch._scaled_mm(a, bt.t(), scale_a=one, scale_b=one, out_dtype=bf))
        th = bench(lambda: gemm.hip_fp8_mm(a, bt, scale_a=one, scale_b=one))
        gemm._fp8_8phase = False
        t2 = bench(lambda: gemm.hip_fp8_mm(a, bt, scale_a=one, scale_b=one))
        gemm._fp8_8phase = True
        th2 = bench(lambda: gemm.hip_fp8_mm(a, bt, scale_a=one, scale_b=one))
        print(f"  fp8 gemm {name}: torch._scaled_mm {tl*1e6:8.1f} us {f1/tl/1e12:6.0f} TF | hip 8-phase "
              f"{th*1e6:8.1f} / {th2*1e6:8.1f} us {f1/min(th, th2)/1e12:6.0f} TF | hip 2-stage {t2*1e6:8.1f} us "
              f"{f1/t2/1e12:6.0f} TF", flush=True)
        m = F8.FP8Meta(F8.E4M3, 16, 0, dev)
        xb = x.detach()
        tc = bench(lambda: m.cast(xb))
        by = M * K * (2 + 1 + 1)
        print(f"  cast+transpose [{M},{K}]: {tc*1e6:8.1f} us {by/tc/1e12:5.2f} TB/s", flush=True)


if __name__ == '__main__':
    main()
