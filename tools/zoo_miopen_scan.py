"""Which paddle.vision.models train (AMP-O2 bf16, default NCHW, one step on a small batch) without a
single library (MIOpen) convolution / batch-norm / pooling kernel: prints the offending kernels per
model."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def library_kernels(fn):
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = {e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA}
    bad = ('miopen', 'igemm', 'naive_conv', 'batchnorm', 'im2col', 'col2im', 'conv_fwd', 'conv_bwd', 'gridwise',
           'winograd', 'pooling', 'xdlops', 'subsample', 'sp3asm', 'mlo')
    return sorted(n[:80] for n in names if any(b in n.lower() for b in bad) and not any(o in n for o in ('pa::', 'pa_')))


def main():
    import paddle
    from paddle.vision import models as M
    cases = [('resnet18', 224), ('resnet50', 224), ('resnext50_32x4d', 224), ('wide_resnet50_2', 224),
             ('vgg16', 224), ('alexnet', 224), ('mobilenet_v1', 224), ('mobilenet_v2', 224),
             ('mobilenet_v3_small', 224), ('mobilenet_v3_large', 224), ('shufflenet_v2_x1_0', 224),
             ('squeezenet1_1', 224), ('densenet121', 224), ('googlenet', 224), ('inception_v3', 299)]
    only = set(sys.argv[1:])
    for name, hw in cases:
        if only and name not in only:
            continue
        if not hasattr(M, name):
            print(f'{name:22s} (not in paddle.vision.models)', flush=True)
            continue
        try:
            paddle.seed(1)
            net = getattr(M, name)(num_classes=10)
            opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=net.parameters(),
                                            multi_precision=True)
            net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
            x = paddle.to_tensor(torch.randn(2, 3, hw, hw, device='cuda').bfloat16())
            y = paddle.to_tensor(torch.randint(0, 10, (2,), device='cuda'))

            def step():
                out = net(x)
                if isinstance(out, (tuple, list)):
                    out = out[0]
                loss = paddle.nn.functional.cross_entropy(out, y)
                loss.backward()
                opt.step()
                opt.clear_grad()
            step()
            bad = library_kernels(step)
            print(f'{name:22s} {"zero library kernels" if not bad else "library: " + "; ".join(bad[:4])}', flush=True)
        except Exception as e:  # noqa: BLE001
            print(f'{name:22s} error: {type(e).__name__}: {str(e)[:150]}', flush=True)


if __name__ == '__main__':
    main()
