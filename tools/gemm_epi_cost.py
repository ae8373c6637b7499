"""Epilogue cost of the schedule-11 GEMM on the GPT-3 1.3B shapes: the same kernel with the
epilogue stores (EPI 0 / 2) vs with its arithmetic only (EPI 10 / 12, csrc/gemm8.hip
pa_gemm8_diag), interleaved rounds in one process, random operands in [-1, 1)."""
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
    from paddle.ops import _native as NT, gemm
    L = NT._load()
    M, dev, bf = 16 * 1024, 'cuda', torch.bfloat16
    rnd = lambda *s: torch.rand(*s, device=dev, dtype=bf) * 2 - 1
    R = int(os.environ.get('ROUNDS', '5'))
    res = {}
    shapes = [('qkv', 2048, 6144), ('out', 2048, 2048), ('fc1', 2048, 8192), ('fc2', 8192, 2048)]
    data = {}
    for name, K, N in shapes:
        data[name] = (rnd(M, K), rnd(N, K), torch.empty(M, N, device=dev, dtype=bf),
                      torch.empty(M, N, device=dev, dtype=bf), rnd(N))
    for r in range(R):
        for name, K, N in shapes:
            a, b, c, aux, bias = data[name]
            epis = (0, 10, 20, 100, 200, 2, 12, 102, 202) if name == 'fc1' else (0, 10, 100, 200)
            for e in epis:
                for st in (0,):
                    fn = lambda e=e: NT.check(L.pa_gemm8_diag(NT.ptr(a), NT.ptr(b), NT.ptr(c), NT.ptr(bias),
                                                              NT.ptr(aux), M, N, K, e, NT.stream()), 'diag')
                    res.setdefault((name, e, st, 2.0 * M * N * K), []).append(timeit(fn))
        # fused MLP epilogues through the production entry (fc2 dgrad x gelu' with the fc1 bias
        # column sums = EPI 4), register-fragment vs LDS-staged epilogue
        a, b, c, aux, bias = data['fc1']
        part = torch.empty(M // 128 * 8192, device=dev, dtype=torch.float32)
        for stg in (0, 1, 3, 4):
            L.pa_gemm8_set_staged_epi(stg)
            res.setdefault(('fc2dgrad-epi4', 4 + 100 * stg, 0, 2.0 * M * 8192 * 2048), []).append(
                timeit(lambda: gemm.mm_epi(a, b.t(), 3, aux, out=c, colsum_part=part)))
            res.setdefault(('fc1fwd-epi2', 2 + 100 * stg, 0, 2.0 * M * 8192 * 2048), []).append(
                timeit(lambda: gemm.mm_epi(a, b.t(), 2, aux, bias=bias, out=c)))
        L.pa_gemm8_set_staged_epi(4)
        print(f'round {r} done', flush=True)
    for (name, e, st, fl), ts in res.items():
        med = statistics.median(ts)
        print(f'{name:4s} epi {e:2d} stagger {st:3d}  med {med * 1e6:7.1f} us  {fl / med / 1e12:6.0f} TF  min {min(ts) * 1e6:7.1f}')


if __name__ == '__main__':
    main()
