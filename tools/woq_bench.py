"""Weight-only int8 / int4 decode GEMM (csrc/woq_gemm.hip) vs the bf16 skinny decode GEMM and the
library on Llama-2-13B layer shapes, M <= 16, random operands; also reports the quantised-weight
streaming bandwidth."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=50):
    """Device time per call: n calls captured in one hipGraph and replayed (eager back-to-back
    launches of these ~10-30 us kernels measure the Python dispatch, not the kernel: the bf16 and
    int8 out-proj GEMMs read 52 vs 26 MB and both timed 15.3 us eagerly)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / (5 * n)


def main():
    import paddle  # noqa: F401
    from paddle.ops import woq, gemm
    from paddle.nn.quant import weight_quantize
    from paddle.ops import _native
    assert _native._load() is not None, _native.load_error
    dev = 'cuda'
    for name, K, N in [('qkv', 5120, 15360), ('out', 5120, 5120), ('ffn1', 5120, 27648), ('ffn2', 13824, 5120)]:
        w = torch.randn(K, N, device=dev) * 0.02
        wb = w.bfloat16()
        q8, s8 = (t._t for t in weight_quantize(paddle.to_tensor(w), 'weight_only_int8'))
        q4, s4 = (t._t for t in weight_quantize(paddle.to_tensor(w), 'weight_only_int4'))
        for M in (1, 8, 16):
            x = torch.randn(M, K, device=dev).bfloat16()
            tb = bench(lambda: gemm.skinny_mm(x, wb))
            tl = bench(lambda: torch.mm(x, wb))
            for fused in ((1, 0) if os.environ.get('WOQ_FUSED_AB') == '1' else (1,)):
                _native.lib.pa_woq_set_fused_finish(fused)
                t8 = bench(lambda: woq.woq_linear(x, q8, s8, 8, 0))
                t4 = bench(lambda: woq.woq_linear(x, q4, s4, 4, 0))
                tag = '' if os.environ.get('WOQ_FUSED_AB') != '1' else (' [fused finish]' if fused else ' [finish kernel]')
                print(f"{name:5s} K={K:5d} N={N:5d} M={M:2d}: bf16 skinny {tb*1e6:7.1f} us ({K*N*2/tb/1e12:4.2f} TB/s) | "
                      f"library {tl*1e6:7.1f} | int8 {t8*1e6:7.1f} us ({K*N/t8/1e12:4.2f} TB/s, {tb/t8:4.2f}x) | "
                      f"int4 {t4*1e6:7.1f} us ({K*N/2/t4/1e12:4.2f} TB/s, {tb/t4:4.2f}x){tag}", flush=True)
            _native.lib.pa_woq_set_fused_finish(1)


def sweep():
    """WOQ_SWEEP=1: K-split target blocks x register stages (pa_woq_tune) on the same shapes."""
    import paddle  # noqa: F401
    from paddle.ops import woq, gemm, _native
    from paddle.nn.quant import weight_quantize
    assert _native._load() is not None, _native.load_error
    L = _native.lib
    dev = 'cuda'
    for name, K, N in [('qkv', 5120, 15360), ('out', 5120, 5120), ('ffn1', 5120, 27648), ('ffn2', 13824, 5120)]:
        w = torch.randn(K, N, device=dev) * 0.02
        wb = w.bfloat16()
        q8, s8 = (t._t for t in weight_quantize(paddle.to_tensor(w), 'weight_only_int8'))
        q4, s4 = (t._t for t in weight_quantize(paddle.to_tensor(w), 'weight_only_int4'))
        for M in (1, 16):
            x = torch.randn(M, K, device=dev).bfloat16()
            tb = bench(lambda: gemm.skinny_mm(x, wb))
            best = {}
            for ct, tgt, nst in [(4, t, 2) for t in (256, 512)] + [(2, t, 2) for t in (128, 256, 512, 1024)]:
                L.pa_woq_set_ct(ct)
                if True:
                    L.pa_woq_tune(tgt, nst)
                    t8 = bench(lambda: woq.woq_linear(x, q8, s8, 8, 0))
                    t4 = bench(lambda: woq.woq_linear(x, q4, s4, 4, 0))
                    print(f"{name:5s} M={M:2d} ct {ct} target {tgt:5d} nst {nst}: int8 {t8*1e6:6.1f} us ({tb/t8:4.2f}x) "
                          f"int4 {t4*1e6:6.1f} us ({tb/t4:4.2f}x)", flush=True)
                    for b, t in ((8, t8), (4, t4)):
                        if b not in best or t < best[b][0]:
                            best[b] = (t, f'{ct}/{tgt}', nst)
            print(f"{name:5s} M={M:2d} bf16 {tb*1e6:6.1f} us | best int8 {best[8][0]*1e6:6.1f} us ({tb/best[8][0]:4.2f}x, "
                  f"target {best[8][1]} nst {best[8][2]}) | best int4 {best[4][0]*1e6:6.1f} us "
                  f"({tb/best[4][0]:4.2f}x, target {best[4][1]} nst {best[4][2]})", flush=True)
    L.pa_woq_tune(-1, 2)
    L.pa_woq_set_ct(0)


if __name__ == '__main__':
    if os.environ.get('WOQ_SWEEP') == '1':
        sweep()
    else:
        main()
