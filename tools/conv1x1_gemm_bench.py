"""1x1 stride-1 ResNet50 convolutions (batch 256, NHWC) as plain GEMMs on the 8-phase MFMA GEMM
(csrc/gemm8.hip) vs the implicit-GEMM conv kernels (csrc/conv.hip): forward, data gradient and
filter gradient, interleaved rounds in one process, random operands.  Prints median us each."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timeit(fn, n=10):
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
    from paddle.ops import conv, gemm, _native
    _native._load()
    dev, bf = 'cuda', torch.bfloat16
    B = 256
    shapes = [(56, 64, 256), (56, 256, 64), (56, 64, 64), (56, 256, 128), (28, 512, 128), (28, 128, 512),
              (28, 512, 256), (14, 1024, 256), (14, 256, 1024), (14, 1024, 512), (7, 2048, 512), (7, 512, 2048)]
    cases = []
    for H, C, Co in shapes:
        x = torch.rand(B, H, H, C, device=dev, dtype=bf) * 2 - 1
        w = torch.rand(Co, C, 1, 1, device=dev, dtype=bf) * 2 - 1
        dy = torch.rand(B, H, H, Co, device=dev, dtype=bf) * 2 - 1
        M = B * H * H
        x2, dy2, w2 = x.view(M, C), dy.view(M, Co), w.view(Co, C)
        tag = f'H{H} C{C}->{Co}'
        fl = 2.0 * M * C * Co
        cases.append((tag, 'fwd', fl, lambda x=x, w=w: conv.conv2d_fwd(x, w, None, (1, 1), (0, 0), (1, 1)),
                      lambda x2=x2, w2=w2: gemm.hip_mm(x2, w2.t()) if gemm.hip_mm_ok(x2, w2.t()) else None))
        cases.append((tag, 'dgrad', fl, lambda dy=dy, w=w, H=H: conv.conv2d_dgrad_classes(dy, w, (H, H), (1, 1), (0, 0), (1, 1)),
                      lambda dy2=dy2, w2=w2: gemm.hip_mm(dy2, w2) if gemm.hip_mm_ok(dy2, w2) else None))
        cases.append((tag, 'wgrad', fl, lambda dy=dy, x=x, w=w: conv.conv2d_wgrad(dy, x, tuple(w.shape), (1, 1), (0, 0), (1, 1)),
                      lambda dy=dy, x=x: conv.conv2d_wgrad_1x1(dy, x)))
    # correctness of the GEMM forms against the conv kernels
    for tag, kind, fl, f0, f1 in cases:
        a, b = f0(), f1()
        if b is None or a is None:
            print(tag, kind, 'gemm form not applicable' if b is None else 'conv form n/a', flush=True)
            continue
        err = float((a.float().reshape(-1) - b.float().reshape(-1)).abs().max())
        ref = float(a.float().abs().max())
        print(f'{tag:16s} {kind:5s} max|conv-gemm| {err:.3g} (|ref| max {ref:.3g})', flush=True)
    R = int(os.environ.get('ROUNDS', '5'))
    res = {}
    for _ in range(R):
        for i, (tag, kind, fl, f0, f1) in enumerate(cases):
            res.setdefault((i, 0), []).append(timeit(f0))
            if f1() is not None:
                res.setdefault((i, 1), []).append(timeit(f1))
    tot = [0.0, 0.0, 0.0]
    for i, (tag, kind, fl, f0, f1) in enumerate(cases):
        t0 = statistics.median(res[(i, 0)])
        t1 = statistics.median(res[(i, 1)]) if (i, 1) in res else float('nan')
        best = min(t0, t1) if t1 == t1 else t0
        tot[0] += t0
        tot[1] += best
        print(f'{tag:16s} {kind:5s}: conv {t0*1e6:7.1f} us ({fl/t0/1e12:4.0f} TF) | gemm {t1*1e6:7.1f} us '
              f'({fl/t1/1e12:4.0f} TF)  {"GEMM" if t1 < t0 else "conv"}', flush=True)
    print(f'sum conv {tot[0]*1e3:.3f} ms, best-of {tot[1]*1e3:.3f} ms')


if __name__ == '__main__':
    main()
