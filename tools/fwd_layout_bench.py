"""Forward GEMM layout A/B for the GPT-3 1.3B step (M = 16 x 1024 tokens).

paddle's Linear weight is [in, out], so y = x @ W + b hands hipBLASLt an N-major B operand.
The dgrad GEMM (dy @ W^T, both operands K-major) runs up to 1.7 PF/s on the same sizes, so
this measures y = x @ (W^T)^T with a per-call transposed copy W^T = [out, in] (the HIP transpose
kernel's time, csrc/act.hip pa_transpose2d, included) against the plain layout, with the committed table and with online
TunableOp tuning of the new layout."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / n


def run(tag):
    M = 16 * 1024
    dev, bf = 'cuda', torch.bfloat16
    shapes = [('qkv', 2048, 6144), ('out', 2048, 2048), ('fc1', 2048, 8192), ('fc2', 8192, 2048)]
    tot_a = tot_b = 0.0
    for name, K, N in shapes:
        x = torch.rand(M, K, device=dev, dtype=bf) * 2 - 1
        w = torch.rand(K, N, device=dev, dtype=bf) * 2 - 1
        b = torch.rand(N, device=dev, dtype=bf)
        wt = w.t().contiguous()
        fl = 2.0 * M * K * N
        ta = bench(lambda: torch.addmm(b, x, w))
        from paddle.ops import gemm
        tt = bench(lambda: gemm.transpose2d(w))
        tb = bench(lambda: torch.addmm(b, x, wt.t()))
        ref = torch.addmm(b, x, w).float()
        err = (torch.addmm(b, x, wt.t()).float() - ref).abs().max().item()
        tot_a += ta
        tot_b += tb + tt
        print(f"[{tag}] {name:4s} K={K} N={N}: x@W {ta*1e6:7.1f} us {fl/ta/1e12:5.0f} TF | "
              f"x@Wt^T {tb*1e6:7.1f} us {fl/tb/1e12:5.0f} TF + transpose {tt*1e6:5.1f} us | maxdiff {err:.3g}",
              flush=True)
        del x, w, b, wt
    print(f"[{tag}] per-layer fwd total: x@W {tot_a*1e3:.3f} ms, x@Wt^T+transpose {tot_b*1e3:.3f} ms", flush=True)


def main():
    from paddle.ops import gemm_tuning
    print('tuned table applied:', gemm_tuning.apply_tuned_db(), flush=True)
    run('table')
    if len(sys.argv) > 1 and sys.argv[1] == 'tune':
        out = os.path.join(os.environ.get('GRAFT_REPO_ROOT', '.'), 'gpurun_out', 'fwd_layout_tuned.csv')
        gemm_tuning.enable_online_tuning(out, max_duration_ms=40, max_iterations=60)
        run('online-tuned')


if __name__ == '__main__':
    main()
