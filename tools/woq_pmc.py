"""Weight-only int8 decode GEMM vs the bf16 skinny GEMM on the Llama-2-13B ffn1 shape (M = 1,
K = 5120, N = 27648), for rocprofv3 --pmc counter passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle
    from paddle.ops import woq, gemm, _native
    from paddle.nn.quant import weight_quantize
    assert _native._load() is not None, _native.load_error
    K, N = 5120, 27648
    w = torch.randn(K, N, device='cuda') * 0.02
    wb = w.bfloat16()
    q8, s8 = (t._t for t in weight_quantize(paddle.to_tensor(w), 'weight_only_int8'))
    x = torch.randn(1, K, device='cuda').bfloat16()
    for _ in range(5):
        gemm.skinny_mm(x, wb)
        woq.woq_linear(x, q8, s8, 8, 0)
    torch.cuda.synchronize()
    print('ok', flush=True)


if __name__ == '__main__':
    main()
