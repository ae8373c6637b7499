"""Interleaved A/B of GEMM schedules 11 (one tile per block) and 12 (persistent, epilogue overlapped
with the next tile's staging) on every GEMM of the GPT-3 1.3B step, in ONE process, random operands
in [-1, 1): R rounds, each round times every (shape, schedule) once; prints median / min us and TF.
Includes the fused-epilogue MLP GEMMs (fc1 forward + GELU, fc2 dgrad * gelu')."""
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
    from paddle.ops import gemm, _native
    L = _native._load()
    M, dev, bf = 16 * 1024, 'cuda', torch.bfloat16
    R = int(os.environ.get('ROUNDS', '5'))
    scheds = [int(s) for s in os.environ.get('SCHEDS', '11,12').split(',')]
    rnd = lambda *s: torch.rand(*s, device=dev, dtype=bf) * 2 - 1
    cases = []
    for name, K, N in [('qkv', 2048, 6144), ('out', 2048, 2048), ('fc1', 2048, 8192), ('fc2', 8192, 2048)]:
        x, wt, dy, w = rnd(M, K), rnd(N, K), rnd(M, N), rnd(K, N)
        fl = 2.0 * M * K * N
        cases.append((f'{name} fwd  x@Wt^T', fl, 'v', lambda x=x, wt=wt: gemm.hip_mm(x, wt.t())))
        cases.append((f'{name} dgrad dy@W^T', fl, 'v', lambda dy=dy, w=w: gemm.hip_mm(dy, w.t())))
    x, wt, b = rnd(M, 2048), rnd(8192, 2048), rnd(8192)
    aux = torch.empty(M, 8192, device=dev, dtype=bf)
    cases.append(('fc1 fwd +gelu (epi2)', 2.0 * M * 2048 * 8192, 'e',
                  lambda: gemm.mm_epi(x, wt.t(), 2, aux, bias=b)))
    dy2, w2 = rnd(M, 2048), rnd(8192, 2048)
    cases.append(('fc2 dgrad *gelu\' (epi3)', 2.0 * M * 2048 * 8192, 'e',
                  lambda: gemm.mm_epi(dy2, w2.t(), 3, aux)))
    h, E = rnd(M, 2048), rnd(50304, 2048)
    cases.append(('lmhead fwd h@E^T', 2.0 * M * 2048 * 50304, 'v', lambda: gemm.hip_mm(h, E.t())))
    res = {}
    for r in range(R):
        for name, fl, kind, fn in cases:
            for s in scheds:
                if kind == 'v':
                    L.pa_gemm_set_variant(s)
                else:
                    L.pa_gemm8_set_epi_sched(s)
                t = timeit(fn, 3 if 'lmhead' in name else 10)
                res.setdefault((name, s), []).append(t)
        L.pa_gemm_set_variant(0)
        L.pa_gemm8_set_epi_sched(11)
        print(f'round {r} done', flush=True)
    for name, fl, kind, fn in cases:
        line = f'{name:26s}'
        for s in scheds:
            ts = res[(name, s)]
            md = statistics.median(ts)
            line += f' | s{s} med {md*1e6:7.1f} us ({fl/md/1e12:5.0f} TF) min {min(ts)*1e6:7.1f}'
        print(line, flush=True)
    # correctness of the persistent epilogue GEMMs vs schedule 11
    outs = {}
    for s in scheds:
        L.pa_gemm8_set_epi_sched(s)
        a2 = torch.empty_like(aux)
        o2 = gemm.mm_epi(x, wt.t(), 2, a2, bias=b)
        o3 = gemm.mm_epi(dy2, w2.t(), 3, a2)
        L.pa_gemm_set_variant(s)
        o0 = gemm.hip_mm(x, wt.t())
        outs[s] = (o2, a2, o3, o0)
    L.pa_gemm8_set_epi_sched(11)
    L.pa_gemm_set_variant(0)
    for s in scheds[1:]:
        d = [float((p.float() - q.float()).abs().max()) for p, q in zip(outs[scheds[0]], outs[s])]
        print(f'max |s{scheds[0]} - s{s}| (gelu, aux, dgrad*aux, plain): {d}', flush=True)


if __name__ == '__main__':
    main()
