"""fp8 cast+transpose kernel modes on the ERNIE / GPT activation shapes (HIP-event timed, median
of 9 x 20 back-to-back casts): 2 = persistent full-tile kernel, 1 = one full tile per block."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from paddle.ops import _native as N  # noqa: E402
from paddle.ops import fp8 as F8  # noqa: E402

assert N._load() is not None, N.load_error
for R, C in [(32768, 768), (32768, 2304), (32768, 3072), (16384, 2048), (768, 768)]:
    x = torch.randn(R, C, device='cuda').to(torch.bfloat16)
    res = {}
    for mode in (1, 2):
        old = N.lib.pa_fp8_set_cast_full(mode)
        m = F8.FP8Meta(torch.float8_e4m3fn, 16, 0, 'cuda')
        for _ in range(5):
            m.cast(x)
        ts = []
        for _ in range(9):  # 20 back-to-back casts per event pair: the host enqueue stays ahead
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(20):
                m.cast(x)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1000 / 20)
        N.lib.pa_fp8_set_cast_full(old)
        ts.sort()
        res[mode] = ts[len(ts) // 2]
    gb = R * C * 4 / 1e9
    print(f"[{R:6d},{C:5d}]  one-tile {res[1]:7.1f} us ({gb / res[1] * 1e6 / 1e3:5.2f} TB/s)  "
          f"persistent {res[2]:7.1f} us ({gb / res[2] * 1e6 / 1e3:5.2f} TB/s)  {res[1] / res[2]:.2f}x", flush=True)
