"""A/B of the software-pipelined flash forward (PA_FA_FWD_SP / pa_flash_set_fwd_sp) vs the classic
kernel at head_dim 64: ERNIE-base (B64 S512 H12, padding mask + dropout 0.1), plain non-causal and
causal.  Prints median forward time and TFLOP/s of each, interleaved rounds."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import paddle  # noqa: E402,F401
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

FA = ops.flash_attn


def timed(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    _native._load()
    cases = []
    B, S, H, D = 64, 512, 12, 64
    q, k, v = (torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16) for _ in range(3))
    keep = torch.ones(B, 1, 1, S, dtype=torch.bool, device='cuda')
    keep[::3, ..., 400:] = False
    fl = 4 * B * H * S * S * D
    cases.append(('ernie mask+drop B64 S512 H12', lambda: FA.flash_attention_ex(q, k, v, mask=keep, dropout=0.1), fl))
    cases.append(('ernie mask      B64 S512 H12', lambda: FA.flash_attention_ex(q, k, v, mask=keep), fl))
    allk = torch.ones(B, 1, 1, S, dtype=torch.bool, device='cuda')
    cases.append(('all-keep mask+drop B64 S512', lambda: FA.flash_attention_ex(q, k, v, mask=allk, dropout=0.1), fl))
    cases.append(('plain           B64 S512 H12', lambda: FA.flash_attention(q, k, v, False), fl))
    B2, S2, H2 = 8, 2048, 16
    q2, k2, v2 = (torch.randn(B2, S2, H2, D, device='cuda', dtype=torch.bfloat16) for _ in range(3))
    fl2 = 4 * B2 * H2 * S2 * S2 * D
    cases.append(('causal          B8 S2048 H16', lambda: FA.flash_attention(q2, k2, v2, True), fl2 / 2))
    cases.append(('non-causal      B8 S2048 H16', lambda: FA.flash_attention(q2, k2, v2, False), fl2))
    res = {}
    with torch.no_grad():
        for rnd in range(3):
            for name, fn, f in cases:
                for sp in (0, 1):
                    _native.lib.pa_flash_set_fwd_sp(sp)
                    res.setdefault((name, sp), []).append(timed(fn))
    # forward + backward of the ERNIE attention (bench shape: an all-keep padding mask + dropout)
    qg, kg, vg = (t.clone().requires_grad_() for t in (q, k, v))
    gout = torch.randn_like(q)

    def fb(mask):
        def f():
            o = FA.flash_attention_ex(qg, kg, vg, mask=mask, dropout=0.1)
            o.backward(gout)
        return f
    for nm, mk in (('fwd+bwd all-keep mask', allk), ('fwd+bwd no mask     ', None), ('fwd+bwd padded mask ', keep)):
        for sp in (0, 1):
            _native.lib.pa_flash_set_fwd_sp(sp)
            t = timed(fb(mk), it=15)
            print(f"{nm} sp={sp}: {t:8.1f} us ({3.5 * fl / t / 1e6:6.0f} TF-equiv)", flush=True)
    for name, fn, f in cases:
        a = sorted(res[(name, 0)])[1]
        b = sorted(res[(name, 1)])[1]
        print(f"{name}: classic {a:8.1f} us ({f / a / 1e6:6.0f} TF) | sp {b:8.1f} us ({f / b / 1e6:6.0f} TF) | "
              f"{a / b:5.2f}x", flush=True)


if __name__ == '__main__':
    main()
