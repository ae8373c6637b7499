"""Debug: forward activations and their gradients, module by module, of resnet50 NCHW vs NHWC
(same weights / input, AMP-O2 bf16); prints the first modules whose outputs or output-gradients
disagree (relative max error), in execution order."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def run(df):
    import paddle
    from paddle.vision.models import resnet50
    paddle.seed(7)
    net = resnet50(num_classes=10, data_format=df)
    opt = paddle.optimizer.Momentum(learning_rate=0.01, momentum=0.9, parameters=net.parameters(),
                                    multi_precision=True)
    net, opt = paddle.amp.decorate(net, opt, level='O2', dtype='bfloat16')
    acts, grads, order = {}, {}, []

    def hook(name):
        def f(layer, inp, out):
            t = out._t if hasattr(out, '_t') else out
            if not isinstance(t, torch.Tensor):
                return
            v = t.detach().float()
            if df == 'NHWC' and v.dim() == 4:
                v = v.permute(0, 3, 1, 2)
            acts[name] = v.clone()
            order.append(name)
            if t.requires_grad:
                def g(gr, name=name):
                    gg = gr.detach().float()
                    if df == 'NHWC' and gg.dim() == 4:
                        gg = gg.permute(0, 3, 1, 2)
                    grads[name] = gg.clone()
                t.register_hook(g)
        return f
    for name, sub in net.named_sublayers():
        if name.count('.') <= 3 and name.startswith(('conv1', 'maxpool', 'layer1.0', 'layer1.1')):
            sub.register_forward_post_hook(hook(name))
        elif name.count('.') <= 2:
            sub.register_forward_post_hook(hook(name))
    from paddle.ops import conv as C, batchnorm as BNM
    hits = []
    orig = C.take_bn_parts

    def spy(x):
        r = orig(x)
        hits.append(r is not None)
        return r
    C.take_bn_parts = spy
    BNM_take = getattr(BNM, 'take_bn_parts', None)
    g = torch.Generator(device='cuda').manual_seed(3)
    img = torch.randn(4, 3, 64, 64, device='cuda', generator=g).bfloat16()
    lab = torch.randint(0, 10, (4,), device='cuda', generator=g)
    xin = paddle.to_tensor(img if df == 'NCHW' else img.permute(0, 2, 3, 1).contiguous())
    loss = paddle.nn.functional.cross_entropy(net(xin), paddle.to_tensor(lab))
    loss.backward()
    C.take_bn_parts = orig
    print(df, 'bn parts hits:', ''.join('1' if h else '0' for h in hits), flush=True)
    return acts, grads, order


def rel(a, b):
    return (a - b).abs().max().item() / (b.abs().max().item() + 1e-12)


def main():
    a1, g1, order = run('NCHW')
    a2, g2, _ = run('NHWC')
    print('forward (execution order):', flush=True)
    for n in order:
        if n in a2 and a1[n].shape == a2[n].shape:
            print(f'  {n:28s} act rel {rel(a1[n], a2[n]):.4f}', flush=True)
    print('backward (output gradients, forward order):', flush=True)
    for n in order:
        if n in g1 and n in g2 and g1[n].shape == g2[n].shape:
            print(f'  {n:28s} grad rel {rel(g1[n], g2[n]):.4f}', flush=True)
        elif n in g1 or n in g2:
            print(f'  {n:28s} grad only in {"NCHW" if n in g1 else "NHWC"}', flush=True)


if __name__ == '__main__':
    main()
