"""Hand-written implicit-GEMM conv2d forward (csrc/conv.hip) vs the storage layer's conv (MIOpen)
on the ResNet50 NHWC bf16 layer shapes at batch 256."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=10):
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


def main():
    import paddle  # noqa: F401
    from paddle.ops import conv, _native
    _native._load()
    B = 256
    shapes = [  # (H, C, Cout, R, stride)
        (56, 64, 64, 1, 1), (56, 64, 64, 3, 1), (56, 64, 256, 1, 1), (56, 256, 64, 1, 1), (56, 256, 128, 1, 1),
        (56, 128, 128, 3, 2), (28, 128, 512, 1, 1), (56, 256, 512, 1, 2), (28, 512, 128, 1, 1), (28, 128, 128, 3, 1),
        (28, 512, 256, 1, 1), (28, 256, 256, 3, 2), (14, 256, 1024, 1, 1), (14, 1024, 256, 1, 1),
        (14, 256, 256, 3, 1), (14, 1024, 512, 1, 1), (14, 512, 512, 3, 2), (7, 512, 2048, 1, 1), (7, 2048, 512, 1, 1),
        (7, 512, 512, 3, 1)]
    tot_h = tot_l = tot_bh = tot_bl = tot_wl = tot_wh = tot_dl = tot_dh = 0.0
    if len(sys.argv) > 1:
        _native.lib.pa_conv2d_wgrad_set_bncap(int(sys.argv[1]))
    if len(sys.argv) > 2:
        _native.lib.pa_conv2d_wgrad_set_wm(int(sys.argv[2]))
    for i, bn in enumerate((64, 128, 256)):  # forward / data-gradient wave layout per Cout tile width
        if len(sys.argv) > 3 + i:
            _native.lib.pa_conv2d_set_wm(bn, int(sys.argv[3 + i]))
    for H, C, Cout, R, s in shapes:
        p = R // 2
        x = torch.randn(B, H, H, C, device='cuda', dtype=torch.bfloat16)
        w = torch.randn(Cout, C, R, R, device='cuda', dtype=torch.bfloat16) * 0.05
        xc = x.permute(0, 3, 1, 2)
        Ho = (H + 2 * p - R) // s + 1
        fl = 2.0 * B * Ho * Ho * Cout * C * R * R
        tl = bench(lambda: torch.nn.functional.conv2d(xc, w, None, s, p))
        th = bench(lambda: conv.conv2d_fwd(x, w, None, (s, s), (p, p), (1, 1)))
        tot_h += th
        tot_l += tl
        # backward: MIOpen data+filter grads vs the hand-written paths (MIOpen where not covered)
        y = conv.conv2d_fwd(x, w, None, (s, s), (p, p), (1, 1))
        dy = torch.randn_like(y)
        dyc = dy.permute(0, 3, 1, 2)
        tbl = bench(lambda: torch.ops.aten.convolution_backward(dyc, xc, w, None, [s, s], [p, p], [1, 1], False,
                                                                [0, 0], 1, [True, True, False]))
        xg = x.detach().requires_grad_()
        wg = w.detach().requires_grad_()
        yy = conv.conv2d_nhwc(xg, wg, None, (s, s), (p, p), (1, 1))
        tbh = bench(lambda: torch.autograd.grad(yy, (xg, wg), dy, retain_graph=True))
        tot_bh += tbh
        tot_bl += tbl
        twl = bench(lambda: torch.ops.aten.convolution_backward(dyc, xc, w, None, [s, s], [p, p], [1, 1], False,
                                                                [0, 0], 1, [False, True, False]))
        twh = bench(lambda: conv.conv2d_wgrad(dy, x, tuple(w.shape), (s, s), (p, p), (1, 1)))
        tdl = bench(lambda: torch.ops.aten.convolution_backward(dyc, xc, w, None, [s, s], [p, p], [1, 1], False,
                                                                [0, 0], 1, [True, False, False]))
        tdh = bench(lambda: conv.conv2d_dgrad_classes(dy, w, (H, H), (s, s), (p, p), (1, 1)))
        tot_dl += tdl
        tot_dh += tdh
        print(f"   dgrad MIOpen {tdl*1e6:7.1f} us {fl/tdl/1e12:4.0f} TF | hip {tdh*1e6:7.1f} us {fl/tdh/1e12:4.0f} TF",
              flush=True)
        tot_wl += twl
        tot_wh += twh
        print(f"   wgrad MIOpen {twl*1e6:7.1f} us {fl/twl/1e12:4.0f} TF | hip {twh*1e6:7.1f} us {fl/twh/1e12:4.0f} TF",
              flush=True)
        print(f"H{H} C{C} Cout{Cout} R{R} s{s}: fwd MIOpen {tl*1e6:7.1f} us {fl/tl/1e12:4.0f} TF | hip {th*1e6:7.1f} us "
              f"{fl/th/1e12:4.0f} TF || bwd MIOpen {tbl*1e6:7.1f} us | ours {tbh*1e6:7.1f} us", flush=True)
    print(f"sum over shapes: fwd MIOpen {tot_l*1e3:.2f} ms, hip {tot_h*1e3:.2f} ms; bwd MIOpen {tot_bl*1e3:.2f} ms, "
          f"ours {tot_bh*1e3:.2f} ms; wgrad MIOpen {tot_wl*1e3:.2f} ms, hip {tot_wh*1e3:.2f} ms; "
          f"dgrad MIOpen {tot_dl*1e3:.2f} ms, hip {tot_dh*1e3:.2f} ms", flush=True)


if __name__ == '__main__':
    main()
