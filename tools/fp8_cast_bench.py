"""fp8 cast + transpose kernel (csrc/fp8_cast.hip pa_fp8_cast_transpose) bandwidth on the ERNIE-base
fp8 step's shapes (32768 tokens; activations 768 / 3072 wide, gradients 768 / 2304 / 3072 wide):
bytes moved = 2 (bf16 read) + 1 (q) + 1 (q^T) per element, device time under hipGraph replay."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def t_ms(fn, it=20, reps=5):
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
    from paddle.ops import fp8, _native
    assert _native._load() is not None
    for fmt, dt in (('e4m3', fp8.E4M3), ('e5m2', fp8.E5M2)):
        for R, C in ((32768, 768), (32768, 2304), (32768, 3072), (768, 3072), (3072, 768)):
            x = torch.randn(R, C, device='cuda').bfloat16()
            meta = fp8.FP8Meta(dt, 16, 0, 'cuda')
            meta.cast(x)
            ms = t_ms(lambda: meta.cast(x))
            gb = R * C * 4 / 1e9
            print(f"{fmt} [{R:6d}, {C:5d}]: {ms * 1e3:7.1f} us  {gb / ms:5.2f} TB/s", flush=True)


if __name__ == '__main__':
    main()
