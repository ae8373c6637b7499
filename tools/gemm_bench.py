"""Per-shape GEMM throughput of the GPT-3 1.3B training step (M = 16 x 1024 tokens) in the three
layouts the step uses (fwd x@W+b, dgrad dy@W^T, wgrad W.grad += x^T@dy), on random operands,
with the committed TunableOp table (set PADDLE_AMD_GEMM_TUNING=0 for the library default)."""
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


def main():
    if os.environ.get('PADDLE_AMD_GEMM_TUNING', '1') != '0':
        from paddle.ops import gemm_tuning
        print('tuned table applied:', gemm_tuning.apply_tuned_db(), flush=True)
    M = 16 * 1024
    dev, bf = 'cuda', torch.bfloat16
    shapes = [('qkv', 2048, 6144), ('out', 2048, 2048), ('fc1', 2048, 8192), ('fc2', 8192, 2048)]
    tot = 0.0
    for name, K, N in shapes:
        x = torch.rand(M, K, device=dev, dtype=bf) * 2 - 1
        w = torch.rand(K, N, device=dev, dtype=bf) * 2 - 1
        b = torch.rand(N, device=dev, dtype=bf)
        dy = torch.rand(M, N, device=dev, dtype=bf) * 2 - 1
        gw = torch.zeros(K, N, device=dev, dtype=bf)
        fl = 2.0 * M * K * N
        t1 = bench(lambda: torch.addmm(b, x, w))
        t2 = bench(lambda: torch.mm(dy, w.t()))
        t3 = bench(lambda: gw.addmm_(x.t(), dy))
        tot += t1 + t2 + t3
        for sp in (2, 4, 8):  # split-M wgrad: one batched GEMM over M/sp slices + a sum of the partials
            xs, ds_ = x.view(sp, M // sp, K).transpose(1, 2), dy.view(sp, M // sp, N)

            def split_wgrad():
                gw.add_(torch.bmm(xs, ds_).sum(0, dtype=torch.float32).to(gw.dtype))
            ts = bench(split_wgrad)
            print(f"      wgrad split-M x{sp}: {ts*1e6:7.1f} us {fl/ts/1e12:5.0f} TF", flush=True)
        print(f"{name:4s} K={K} N={N}: fwd {t1*1e6:7.1f} us {fl/t1/1e12:5.0f} TF | dgrad {t2*1e6:7.1f} us "
              f"{fl/t2/1e12:5.0f} TF | wgrad {t3*1e6:7.1f} us {fl/t3/1e12:5.0f} TF", flush=True)
        del x, w, b, dy, gw
    print(f"per-layer GEMM total {tot*1e3:.3f} ms -> x24 = {tot*24e3:.1f} ms", flush=True)
    V = 50304
    h = torch.rand(M, 2048, device=dev, dtype=bf) * 2 - 1
    E = torch.rand(V, 2048, device=dev, dtype=bf) * 2 - 1
    dl = torch.rand(M, V, device=dev, dtype=bf) * 2 - 1
    gE = torch.zeros(V, 2048, device=dev, dtype=bf)
    fl = 2.0 * M * 2048 * V
    t1 = bench(lambda: torch.matmul(h, E.t()), 5)
    t2 = bench(lambda: torch.mm(dl, E), 5)
    t3 = bench(lambda: gE.addmm_(dl.t(), h), 5)
    print(f"lmhead V={V}: fwd {t1*1e6:7.1f} us {fl/t1/1e12:5.0f} TF | dgrad {t2*1e6:7.1f} us {fl/t2/1e12:5.0f} TF | "
          f"wgrad {t3*1e6:7.1f} us {fl/t3/1e12:5.0f} TF", flush=True)
    del h, E, dl, gE
    for n in (4096, 8192):
        a = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
        bb = torch.rand(n, n, device=dev, dtype=bf) * 2 - 1
        t = bench(lambda: torch.mm(a, bb))
        tt = bench(lambda: torch.mm(a, bb.t()))
        print(f"square {n}: NN {2*n**3/t/1e12:.0f} TF, NT {2*n**3/tt/1e12:.0f} TF", flush=True)


if __name__ == '__main__':
    main()
