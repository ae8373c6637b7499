"""Fused bias+GELU(tanh) forward (csrc/act.hip bias_act_fwd_2d) on the GPT-3 1.3B fc1 output
[16384, 8192] bf16: A/B of the launch shape (target workgroups x rows in flight per thread)
against a plain device copy of the same bytes (read x, write y) as the HBM roofline."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / it


def main():
    import paddle  # noqa: F401
    from paddle.ops import _native, act
    _native._load()
    rows, cols = 16384, 8192
    x = torch.randn(rows, cols, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(cols, device='cuda', dtype=torch.bfloat16)
    y = torch.empty_like(x)
    nbytes = 2 * x.numel() * 2
    t = timeit(lambda: y.copy_(x))
    print(f"copy (roofline)            : {t*1e6:7.1f} us  {nbytes / t / 1e12:5.2f} TB/s", flush=True)
    ref = torch.nn.functional.gelu(x.float() + b.float(), approximate='tanh')
    best = None
    for blocks in (1024, 2048, 4096, 8192):
        for unroll in (2, 4, 8):
            _native.lib.pa_act_fwd_tune(blocks, unroll)
            out = act.gelu(x, approximate=True, bias=b)
            err = (out.float() - ref).abs().max().item()
            t = timeit(lambda: act.gelu(x, approximate=True, bias=b))
            print(f"blocks={blocks:5d} unroll={unroll}: {t*1e6:7.1f} us  {nbytes / t / 1e12:5.2f} TB/s  "
                  f"maxerr {err:.3g}", flush=True)
            if best is None or t < best[0]:
                best = (t, blocks, unroll)
    print(f"best: blocks={best[1]} unroll={best[2]} {best[0]*1e6:.1f} us", flush=True)
    _native.lib.pa_act_fwd_tune(8192, 2)

    # backward: dx = dy * gelu'(x + b) and dbias = colsum(dx) in one column-blocked kernel
    dy = torch.randn_like(x)
    dx = torch.empty_like(x)
    db = torch.zeros(cols, device='cuda', dtype=torch.float32)
    xr = (x.float() + b.float()).requires_grad_(True)
    torch.nn.functional.gelu(xr, approximate='tanh').backward(dy.float())
    nb = 3 * x.numel() * 2
    for blocks in (1024, 2048, 4096, 8192):
        _native.lib.pa_act_cs_tune(blocks)
        nparts = _native.lib.pa_colsum_nparts(rows, cols, _native.dtcode(x.dtype))
        part = torch.empty(nparts * cols, device='cuda', dtype=torch.float32)

        def bwd():
            _native.check(_native.lib.pa_bias_act_bwd_dbias(1, _native.ptr(dy), _native.ptr(x), _native.ptr(b),
                                                            _native.ptr(dx), _native.ptr(part), _native.ptr(db),
                                                            _native.dtcode(db.dtype), 0, rows, cols,
                                                            _native.dtcode(x.dtype), _native.stream()), 'bwd')
        bwd()
        torch.cuda.synchronize()
        edx = (dx.float() - xr.grad).abs().max().item()
        edb = ((db - xr.grad.sum(0)).abs().max() / xr.grad.sum(0).abs().max()).item()
        t = timeit(bwd)
        print(f"bwd blocks={blocks:5d} (nparts {nparts}): {t*1e6:7.1f} us  {nb / t / 1e12:5.2f} TB/s  "
              f"dx maxerr {edx:.3g} dbias relerr {edb:.3g}", flush=True)
    _native.lib.pa_act_cs_tune(1024)


if __name__ == '__main__':
    main()
