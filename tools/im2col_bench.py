"""Isolated timing of the stem im2col kernel (csrc/conv.hip pa_im2col_nhwc) vs a plain fill of
the same output and a copy of the input, ResNet50 stem shape (256 x 224 x 224 x 3 -> [802816, 192])."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddle  # noqa: E402,F401
from paddle.ops import _native as N  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    N._load()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    x = torch.randn(B, 224, 224, 3, device='cuda').to(torch.bfloat16)
    M, Kp = B * 112 * 112, 192
    out = torch.empty(M, Kp, dtype=torch.bfloat16, device='cuda')

    def im2col():
        N.check(N.lib.pa_im2col_nhwc(N.ptr(x), N.ptr(out), B, 224, 224, 3, 7, 7, 2, 2, 3, 3, 1, 1, 112, 112, Kp,
                                     N.stream()), 'im2col')
    im2col()
    torch.cuda.synchronize()
    ref = torch.nn.functional.unfold(x[:1].float().permute(0, 3, 1, 2), 7, padding=3, stride=2)  # [1, 147, L] (c, r, s)
    r0 = ref[0].t()[:5].reshape(5, 3, 7, 7).permute(0, 2, 3, 1).reshape(5, 7, 21)
    got = out[:5, :168].float().reshape(5, 7, 24)[:, :, :21]
    print("max |im2col - unfold| on 5 rows:", (got - r0).abs().max().item())
    t_i = timeit(im2col)
    t_f = timeit(lambda: out.fill_(1.0))
    y = torch.empty_like(x)
    t_c = timeit(lambda: y.copy_(x))
    gb = out.numel() * 2 / 1e9
    print(f"im2col {t_i:.1f} us ({gb / t_i * 1e3:.2f} TB/s of output), fill {t_f:.1f} us ({gb / t_f * 1e3:.2f} TB/s), "
          f"input copy {t_c:.1f} us")


if __name__ == '__main__':
    main()
