"""Times csrc/flash_attn.hip fwd / fwd+bwd against torch SDPA (library) on GPT-1.3B shapes."""
import sys
import os
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import paddle  # noqa: F401
from paddle import ops
from paddle.ops import _native
_native._load()


def timeit_plain(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def timeit(fn, n=10):
    """GPU time per call: n calls captured in one HIP graph, replayed and timed with events
    (host launch overhead excluded)."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
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
    if os.environ.get('FA_DS_AB') == '1':  # recompute backward vs materialised-dS backward
        for on in (False, True):
            ops.flash_attn.set_ds_backward(on)
            print(f"-- dS backward {'on' if on else 'off'}", flush=True)
            run()
        return
    for var in [int(x) for x in os.environ.get('FA_VARIANTS', '1').split(',')]:
        _native.lib.pa_flash_set_bwd_variant(var)
        print(f"-- backward variant {var}", flush=True)
        run()


def run():
    shapes = [(16, 1024, 16, 128, True), (4, 4096, 16, 128, True), (16, 1024, 16, 128, False), (8, 2048, 32, 64, True)]
    if os.environ.get('FA_SHAPES') == 'wide':  # native head_dim 96 / 256 (csrc/flash_attn_wide.hip)
        shapes = [(8, 2048, 16, 96, True), (8, 2048, 16, 96, False), (4, 2048, 8, 256, True), (4, 2048, 8, 256, False)]
    for (B, S, H, D, causal) in shapes:
        qkv = torch.randn(B, S, 3, H, D, device='cuda', dtype=torch.bfloat16, requires_grad=True)
        flops = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
        o = ops.flash_attn.flash_attention_packed(qkv, causal)
        g = torch.randn_like(o)
        tf = timeit(lambda: ops.flash_attn.flash_attention_packed(qkv.detach(), causal))
        tfb = timeit_plain(lambda: ops.flash_attn.flash_attention_packed(qkv, causal).backward(g))
        q, k, v = (qkv[:, :, i].transpose(1, 2).detach().clone().requires_grad_() for i in range(3))
        ts = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q.detach(), k.detach(), v.detach(),
                                                                              is_causal=causal))
        gt = g.transpose(1, 2)
        tsb = timeit_plain(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=causal).backward(gt))
        print(f"B{B} S{S} H{H} D{D} causal={causal}: ours fwd {tf*1e3:.3f} ms ({flops/tf/1e12:.0f} TF) "
              f"fwd+bwd {tfb*1e3:.3f} ms ({3.5*flops/tfb/1e12:.0f} TF) | sdpa fwd {ts*1e3:.3f} ms "
              f"({flops/ts/1e12:.0f} TF) fwd+bwd {tsb*1e3:.3f} ms ({3.5*flops/tsb/1e12:.0f} TF)", flush=True)


if __name__ == '__main__':
    main()
