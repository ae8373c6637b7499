"""A/B of the flash-attention block order (pa_flash_set_pair_group: 0 = longest-first over the whole
grid, G > 0 = groups of G (head, batch) pairs per XCD) on the GPT-3 1.3B attention shape, in
interleaved rounds in one process."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddle  # noqa: F401,E402
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

lib = _native._load()
FA = ops.flash_attn


def timeit(fn, n=20):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    groups = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else '0,1,2,4,8,16').split(',')]
    res = {}
    for (B, S, H, D) in [(16, 1024, 16, 128), (8, 2048, 16, 128)]:
        q, k, v = (torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
        g = torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16)
        for rnd in range(3):
            for G in groups:
                lib.pa_flash_set_pair_group(G)
                with torch.no_grad():
                    tf = timeit(lambda: FA.flash_attention(q, k, v, True))
                tfb = timeit(lambda: FA.flash_attention(q, k, v, True).backward(g))
                res.setdefault((B, S, G), []).append((tf, tfb - tf))
    lib.pa_flash_set_pair_group(0)
    for (B, S, G), v in sorted(res.items()):
        f = sorted(x[0] for x in v)[len(v) // 2]
        b = sorted(x[1] for x in v)[len(v) // 2]
        print(f"B{B} S{S} G={G:2d}: fwd {f:.3f} ms  bwd {b:.3f} ms  (median of {len(v)})", flush=True)


if __name__ == '__main__':
    main()
