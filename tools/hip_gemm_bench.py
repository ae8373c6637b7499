"""Hand-written MFMA GEMM (csrc/gemm.hip) vs hipBLASLt (torch + committed TunableOp table) on the
GPT-3 1.3B step's GEMM shapes (M = 16 x 1024 tokens) in the three layouts the step uses, random
operands.  Prints us and TF/s per (shape, layout, splitk)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=20):
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


VARIANTS = [int(v) for v in os.environ.get('GEMM_VARIANTS', '1,3').split(',')]


def main():
    import paddle  # noqa: F401
    from paddle.ops import gemm, gemm_tuning, _native
    _native._load()
    print('tuned table applied:', gemm_tuning.apply_tuned_db(), flush=True)
    M = 16 * 1024
    dev, bf = 'cuda', torch.bfloat16
    shapes = [('qkv', 2048, 6144), ('out', 2048, 2048), ('fc1', 2048, 8192), ('fc2', 8192, 2048)]
    if len(sys.argv) > 1 and sys.argv[1] == 'fp8':
        e4 = torch.float8_e4m3fn
        one = torch.ones((), device=dev)
        for name, K, N in [('qkv', 2048, 6144), ('out', 2048, 2048), ('fc1', 2048, 8192), ('fc2', 8192, 2048),
                           ('sq8k', 8192, 8192)]:
            a = (torch.rand(M, K, device=dev) * 2 - 1).to(e4)
            w = (torch.rand(N, K, device=dev) * 2 - 1).to(e4)
            fl = 2.0 * M * K * N
            tl = bench(lambda: torch._scaled_mm(a, w.t(), scale_a=one, scale_b=one, out_dtype=bf))
            th = bench(lambda: gemm.hip_fp8_mm(a, w, scale_a=one, scale_b=one))
            print(f"fp8 {name} M={M} K={K} N={N}: torch._scaled_mm {tl*1e6:8.1f} us {fl/tl/1e12:6.0f} TF | "
                  f"hip {th*1e6:8.1f} us {fl/th/1e12:6.0f} TF", flush=True)
        return
    if len(sys.argv) > 1 and sys.argv[1] == 'lmhead':
        V, Hd = 50304, 2048
        h = torch.rand(M, Hd, device=dev, dtype=bf) * 2 - 1
        E = torch.rand(V, Hd, device=dev, dtype=bf) * 2 - 1
        dl = torch.rand(M, V, device=dev, dtype=bf) * 2 - 1
        gE = torch.zeros(V, Hd, device=dev, dtype=bf)
        fl = 2.0 * M * Hd * V
        for lay, lib, mine in (('fwd h@E^T', lambda: torch.mm(h, E.t()), lambda: gemm.hip_mm(h, E.t())),
                               ('dgrad dl@E', lambda: torch.mm(dl, E), lambda: gemm.hip_mm(dl, E)),
                               ('wgrad dl^T@h', lambda: gE.addmm_(dl.t(), h),
                                lambda: gemm.hip_mm(dl.t(), h, out=gE, beta=1.0))):
            tl, th = bench(lib, 5), bench(mine, 5)
            print(f"lmhead {lay:14s}: hipBLASLt {tl*1e6:8.1f} us {fl/tl/1e12:6.0f} TF | hip {th*1e6:8.1f} us "
                  f"{fl/th/1e12:6.0f} TF", flush=True)
        return
    if len(sys.argv) > 1 and sys.argv[1] == 'square':
        shapes = [('sq4k', 4096, 4096), ('sq8k', 8192, 8192)]
        M = None
    for name, K, N in shapes:
        m = M or K
        x = torch.rand(m, K, device=dev, dtype=bf) * 2 - 1
        w = torch.rand(K, N, device=dev, dtype=bf) * 2 - 1
        dy = torch.rand(m, N, device=dev, dtype=bf) * 2 - 1
        gw = torch.zeros(K, N, device=dev, dtype=bf)
        fl = 2.0 * m * K * N
        rows = []
        for lay, lib, mine in (
                ('fwd  x@W', lambda: torch.mm(x, w), lambda s: gemm.hip_mm(x, w, splitk=s)),
                ('dgrad dy@W^T', lambda: torch.mm(dy, w.t()), lambda s: gemm.hip_mm(dy, w.t(), splitk=s)),
                ('wgrad += x^T@dy', lambda: gw.addmm_(x.t(), dy),
                 lambda s: gemm.hip_mm(x.t(), dy, out=gw, beta=1.0, splitk=s))):
            tl = bench(lib)
            best = None
            for var in VARIANTS:
                _native.lib.pa_gemm_set_variant(var)
                for s in (1, 2, 4):
                    kk = K if not lay.startswith('wgrad') else m
                    if kk % (64 * s) or (s > 1 and not lay.startswith('wgrad')):
                        continue
                    t = bench(lambda: mine(s))
                    rows.append(f"   hip v{var} splitk={s}: {t*1e6:8.1f} us {fl/t/1e12:6.0f} TF")
                    best = t if best is None else min(best, t)
            print(f"{name} K={K} N={N} {lay:16s}: hipBLASLt {tl*1e6:8.1f} us {fl/tl/1e12:6.0f} TF | "
                  f"hip best {best*1e6:8.1f} us {fl/best/1e12:6.0f} TF", flush=True)
            for r in rows:
                print(r, flush=True)
            rows = []
        del x, w, dy, gw


if __name__ == '__main__':
    main()
