"""Weight-only decode GEMM kernels (int8 / int4, M = 1) on the 13B layer shapes, for
rocprofv3 --kernel-trace --stats: per-kernel device time of woq_kernel and woq_finish."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle
    from paddle.ops import woq, _native
    from paddle.nn.quant import weight_quantize
    assert _native._load() is not None, _native.load_error
    M = int(os.environ.get('WOQ_M', '1'))
    for name, (K, N) in {'qkv': (5120, 15360), 'out': (5120, 5120), 'ffn1': (5120, 27648),
                         'ffn2': (13824, 5120)}.items():
        w = torch.randn(K, N, device='cuda') * 0.02
        x = torch.randn(M, K, device='cuda').bfloat16()
        for algo, bits in (('weight_only_int8', 8), ('weight_only_int4', 4)):
            q, s = (t._t for t in weight_quantize(paddle.to_tensor(w), algo))
            for _ in range(20):
                woq.woq_linear(x, q, s, bits, 0)
        torch.cuda.synchronize()
        print(name, 'ok', flush=True)


if __name__ == '__main__':
    main()
