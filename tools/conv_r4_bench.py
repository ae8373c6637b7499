"""Round-4 conv kernels vs the library (MIOpen through torch), bf16:
* the ResNet50 stem forward (256x224x224x3 -> 64, 7x7/2) on csrc/conv_stem.hip,
* MobileNet-style depthwise 3x3 forward / data gradient / filter gradient on csrc/dwconv.hip,
* a default-NCHW resnet50() O2 training step vs the NHWC model (img/s)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def timeit(fn, n=10, rounds=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n * 1e3)
    return statistics.median(ts)


def main():
    import paddle
    from paddle.ops import conv, _native
    _native._load()
    dev, bf = 'cuda', torch.bfloat16
    # stem
    x = torch.randn(256, 224, 224, 3, device=dev, dtype=bf)
    w = (0.1 * torch.randn(64, 3, 7, 7, device=dev)).to(bf)
    xc = x.permute(0, 3, 1, 2)
    t_ours = timeit(lambda: conv.conv2d_fwd_stem(x, w, None, (2, 2), (3, 3)))
    t_lib = timeit(lambda: torch.nn.functional.conv2d(xc, w, None, 2, 3))
    y = conv.conv2d_fwd_stem(x, w, None, (2, 2), (3, 3))
    print(f'stem fwd 256x224x224x3->64 7x7/2: hip {t_ours:8.1f} us  library {t_lib:8.1f} us  '
          f'({y.numel() * 2 / t_ours / 1e6:.2f} TB/s output)', flush=True)
    # depthwise (MobileNetV2-like shapes at batch 128)
    for (H, C, s) in [(112, 32, 1), (112, 96, 2), (56, 144, 1), (28, 192, 1), (14, 384, 1), (14, 576, 1), (7, 960, 1)]:
        x = torch.randn(128, H, H, C, device=dev, dtype=bf)
        wd = (0.3 * torch.randn(C, 1, 3, 3, device=dev)).to(bf)
        xc = x.permute(0, 3, 1, 2)  # channels-last strides for the library
        y = conv.dwconv2d_nhwc(x, wd, None, (s, s), (1, 1), (1, 1))
        dy = torch.randn_like(y)
        tf = timeit(lambda: conv.dwconv2d_nhwc(x, wd, None, (s, s), (1, 1), (1, 1)))
        tl = timeit(lambda: torch.nn.functional.conv2d(xc, wd, None, s, 1, 1, C))
        xg, wg = x.clone().requires_grad_(), wd.clone().requires_grad_()
        yy = conv.dwconv2d_nhwc(xg, wg, None, (s, s), (1, 1), (1, 1))
        tb = timeit(lambda: torch.autograd.grad(yy, (xg, wg), dy, retain_graph=True))
        xcg, wcg = xc.detach().clone().requires_grad_(), wd.clone().requires_grad_()
        yl = torch.nn.functional.conv2d(xcg, wcg, None, s, 1, 1, C)
        dyl = dy.permute(0, 3, 1, 2)
        tbl = timeit(lambda: torch.autograd.grad(yl, (xcg, wcg), dyl, retain_graph=True))
        print(f'dw3x3 128x{H}x{H}x{C} s{s}: fwd hip {tf:7.1f} lib {tl:7.1f} us | bwd hip {tb:7.1f} lib {tbl:7.1f} us',
              flush=True)
    # resnet50 NCHW (default) vs NHWC step
    from paddle.vision.models import resnet50
    for df in ('NHWC', 'NCHW'):
        paddle.seed(0)
        net = resnet50(data_format=df)
        opt = paddle.optimizer.Momentum(learning_rate=0.1, momentum=0.9, parameters=net.parameters(),
                                        multi_precision=True)
        net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
        B = 256
        img = torch.randn(B, 3, 224, 224, device=dev).to(bf)
        xin = paddle.to_tensor(img if df == 'NCHW' else img.permute(0, 2, 3, 1).contiguous())
        lab = paddle.to_tensor(torch.randint(0, 1000, (B,), device=dev))

        def step():
            loss = paddle.nn.functional.cross_entropy(net(xin), lab)
            loss.backward()
            opt.step()
            opt.clear_grad()

        t = timeit(step, n=5, rounds=3)
        print(f'resnet50 {df} O2 bf16 batch {B}: {t / 1e3:7.2f} ms/step  {B / (t / 1e6):8.0f} img/s', flush=True)


if __name__ == '__main__':
    main()
