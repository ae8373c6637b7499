"""Run GEMMs of the GPT-3 1.3B fc1 shapes once each (after warmup) for rocprofv3 --pmc counter
collection: the hand-written kernel (schedule given by GEMM_VARIANT, default 8) in the three
layouts, and hipBLASLt on the same operands (tools/gpu_r2_pmc.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle  # noqa: F401
    from paddle.ops import gemm, _native
    _native._load()
    _native.lib.pa_gemm_set_variant(int(os.environ.get('GEMM_VARIANT', '8')))
    M, K, N = 16384, 2048, 8192
    x = torch.rand(M, K, device='cuda', dtype=torch.bfloat16) * 2 - 1
    w = torch.rand(K, N, device='cuda', dtype=torch.bfloat16) * 2 - 1
    dy = torch.rand(M, N, device='cuda', dtype=torch.bfloat16) * 2 - 1
    gw = torch.zeros(K, N, device='cuda', dtype=torch.bfloat16)
    wt = w.t().contiguous()
    for it in range(4):
        gemm.hip_mm(x, w)           # fwd: A k-major, B n-major (tr reads)
        gemm.hip_mm(dy, w.t())      # dgrad: both k-major
        gemm.hip_mm(x.t(), dy, out=gw, beta=1.0)  # wgrad: both m/n-major
        if os.environ.get('GEMM_LIB', '1') == '1':
            torch.mm(dy, w.t())     # hipBLASLt dgrad
            torch.mm(x, wt.t())     # hipBLASLt fwd on the K-major weight copy
    torch.cuda.synchronize()
    print('ok', flush=True)


if __name__ == '__main__':
    main()
