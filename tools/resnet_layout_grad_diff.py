"""Debug: one AMP-O2 bf16 forward/backward of resnet50(data_format='NCHW') vs 'NHWC' with the same
weights and input; prints the loss and the parameters whose gradients differ most (relative)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def grads(df, env=None):
    import paddle
    from paddle.vision.models import resnet50
    from paddle.vision.models import resnet as R
    if env:
        for k, v in env.items():
            setattr(R, k, v)
    paddle.seed(7)
    net = resnet50(num_classes=10, data_format=df)
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=net.parameters(),
                                    multi_precision=True)
    net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
    g = torch.Generator(device='cuda').manual_seed(3)
    img = torch.randn(4, 3, 64, 64, device='cuda', generator=g).bfloat16()
    lab = torch.randint(0, 10, (4,), device='cuda', generator=g)
    xin = paddle.to_tensor(img if df == 'NCHW' else img.permute(0, 2, 3, 1).contiguous())
    loss = paddle.nn.functional.cross_entropy(net(xin), paddle.to_tensor(lab))
    loss.backward()
    out = {}
    for n, p in net.named_parameters():
        gr = p.grad
        out[n] = None if gr is None else gr._t.float().clone()
    return float(loss), out


def main():
    for sink in (True, False):
        env = {'RESIDUAL_GRAD_SINK': sink}
        l1, g1 = grads('NCHW', env)
        l2, g2 = grads('NHWC', env)
        print(f'RESIDUAL_GRAD_SINK={sink}: loss NCHW {l1:.5f} NHWC {l2:.5f}', flush=True)
        rows = []
        for n in g1:
            a, b = g1[n], g2.get(n)
            if a is None or b is None:
                rows.append((float('inf'), n, 'missing', a is None, b is None))
                continue
            d = (a - b).abs().max().item() / (b.abs().max().item() + 1e-12)
            rows.append((d, n, tuple(a.shape)))
        rows.sort(key=lambda r: -r[0])
        for r in rows[:12]:
            print('  ', r, flush=True)


if __name__ == '__main__':
    main()
