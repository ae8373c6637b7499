"""NHWC max pool 3x3/s2/p1 on the ResNet50 stem activation (256 x 112 x 112 x 64 bf16):
csrc/pool.hip vs torch (library) forward + backward."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as TF


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
    return e0.elapsed_time(e1) / n * 1e3


def main():
    from paddle.ops import pool
    x = torch.randn(256, 112, 112, 64, device='cuda').bfloat16().requires_grad_()
    dy = torch.randn(256, 56, 56, 64, device='cuda').bfloat16()
    xc = x.detach().permute(0, 3, 1, 2).requires_grad_()  # channels-last view, as the model runs it

    def hip_fb():
        y = pool.max_pool2d_nhwc(x, (3, 3), (2, 2), (1, 1))
        y.backward(dy)

    def lib_fb():
        y = TF.max_pool2d(xc, 3, 2, 1)
        y.backward(dy.permute(0, 3, 1, 2))
    th = bench(lambda: pool.max_pool2d_nhwc(x.detach(), (3, 3), (2, 2), (1, 1)))
    tl = bench(lambda: TF.max_pool2d(xc.detach(), 3, 2, 1))
    print(f"fwd: hip {th:7.1f} us | torch {tl:7.1f} us", flush=True)
    th = bench(hip_fb)
    tl = bench(lib_fb)
    print(f"fwd+bwd: hip {th:7.1f} us | torch {tl:7.1f} us", flush=True)


if __name__ == '__main__':
    main()
