"""Run the hand-written GEMM on the fc1 shapes (fwd, dgrad, wgrad) a few times each, for
rocprofv3 --pmc counter collection (tools/gpu_check23.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle  # noqa: F401
    from paddle.ops import gemm, _native
    _native._load()
    M, K, N = 16384, 2048, 8192
    x = torch.rand(M, K, device='cuda', dtype=torch.bfloat16) * 2 - 1
    w = torch.rand(K, N, device='cuda', dtype=torch.bfloat16) * 2 - 1
    dy = torch.rand(M, N, device='cuda', dtype=torch.bfloat16) * 2 - 1
    gw = torch.zeros(K, N, device='cuda', dtype=torch.bfloat16)
    for _ in range(3):
        gemm.hip_mm(x, w)           # fwd: A k-major, B n-major (tr reads)
        gemm.hip_mm(dy, w.t())      # dgrad: both k-major
        gemm.hip_mm(x.t(), dy, out=gw, beta=1.0)  # wgrad: both m/n-major
    torch.cuda.synchronize()
    print('ok', flush=True)


if __name__ == '__main__':
    main()
