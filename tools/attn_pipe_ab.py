"""A/B of the flash-attention LDS double buffering (forward PIPE switch, backward variant 4 vs 3)
on the GPT-3 1.3B attention shape (B16 S1024 H16 D128 causal), plain and with dropout 0.1,
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
    B, S, H, D = 16, 1024, 16, 128
    q, k, v = (torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    g = torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16)
    res = {}
    for rnd in range(3):
        for drop in (0.0, 0.1):
            f = (lambda: FA.flash_attention(q, k, v, True)) if drop == 0 else \
                (lambda: FA.flash_attention_ex(q, k, v, True, dropout=0.1))
            for pipe in (0, 1):
                lib.pa_flash_set_fwd_pipe(pipe)
                with torch.no_grad():
                    tf = timeit(f)
                res.setdefault(('fwd', drop, pipe), []).append(tf)
            lib.pa_flash_set_fwd_pipe(0)
            for var in (3, 4):
                lib.pa_flash_set_bwd_variant(var)
                with torch.no_grad():
                    tf = timeit(f)
                tfb = timeit(lambda: f().backward(g))
                res.setdefault(('bwd', drop, var), []).append(tfb - tf)
    lib.pa_flash_set_bwd_variant(0)
    for key, v in sorted(res.items()):
        med = sorted(v)[len(v) // 2]
        print(f"{key[0]} dropout={key[1]} {'pipe' if key[0] == 'fwd' else 'variant'}={key[2]}: {med:.3f} ms "
              f"(median of {len(v)}: {' '.join(f'{x:.3f}' for x in v)})", flush=True)


if __name__ == '__main__':
    main()
