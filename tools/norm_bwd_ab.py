"""LayerNorm backward at narrow rows: the one-wave-per-row kernel vs the block-per-row kernel
(pa_norm_set_bwd_wave A/B), HIP-event timed over 20 back-to-back backward passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from paddle import ops  # noqa: E402
from paddle.ops import _native as N  # noqa: E402

assert N._load() is not None, N.load_error
for rows, cols in [(32768, 768), (16384, 1024), (65536, 512), (16384, 2048)]:
    x = torch.randn(rows, cols, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    w = torch.ones(cols, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    b = torch.zeros(cols, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(rows, cols, device='cuda', dtype=torch.bfloat16)
    res = {}
    for mode in (0, 1):
        old = N.lib.pa_norm_set_bwd_wave(mode)
        y = ops.norm.layer_norm(x, w, b, 1e-5)
        for _ in range(3):
            torch.autograd.grad(y, (x, w, b), g, retain_graph=True)
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(20):
            torch.autograd.grad(y, (x, w, b), g, retain_graph=True)
        e.record()
        e.synchronize()
        res[mode] = a.elapsed_time(e) * 1000 / 20
        N.lib.pa_norm_set_bwd_wave(old)
    gb = rows * cols * 2 * 3 / 1e9
    print(f"[{rows:6d},{cols:5d}] block-per-row {res[0]:7.1f} us ({gb / res[0] * 1e3:5.2f} TB/s)  "
          f"wave-per-row {res[1]:7.1f} us ({gb / res[1] * 1e3:5.2f} TB/s)  {res[0] / res[1]:.2f}x", flush=True)
