"""Weight-gradient GEMM (gw += x^T @ dy, both m/n-contiguous) split-K A/B on the ERNIE-base shapes
(32768 tokens: outputs 768 x 2304 / 768 / 3072 and 3072 x 768 — 9..36 256x256 tiles) and the
GPT-3 1.3B out-projection (16384 tokens, 2048 x 2048): device time under hipGraph replay,
including the split-K reduce."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def t_ms(fn, it=10, reps=5):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(it):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (it * reps)


def main():
    import paddle  # noqa: F401
    from paddle.ops import gemm, _native
    assert _native._load() is not None
    for T, Kin, Nout in ((32768, 768, 2304), (32768, 768, 768), (32768, 768, 3072), (32768, 3072, 768),
                         (16384, 2048, 2048), (16384, 2048, 6144)):
        x = torch.randn(T, Kin, device='cuda').bfloat16()
        dy = torch.randn(T, Nout, device='cuda').bfloat16()
        gw = torch.zeros(Kin, Nout, device='cuda').bfloat16()
        res = []
        for s in (1, 2, 4, 7, 8, 9, 16):
            if not gemm.hip_mm_ok(x.t(), dy, s):
                continue
            ms = t_ms(lambda: gemm.hip_mm(x.t(), dy, out=gw, beta=1.0, splitk=s))
            res.append(f"s{s} {ms * 1e3:6.1f} us ({2 * T * Kin * Nout / ms / 1e9:5.0f} TF)")
        auto = gemm._splitk_for(Kin, Nout, T)
        print(f"[{Kin:4d} x {Nout:4d}] K={T}: " + " | ".join(res) + f"  (auto s{auto})", flush=True)


if __name__ == '__main__':
    main()
