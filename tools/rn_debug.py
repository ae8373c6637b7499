"""ResNet50 NHWC O2: gradients with the fused HIP batch-norm vs the unfused path (same init/input)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import paddle
from paddle.vision.models import resnet50
from paddle.ops import batchnorm

paddle.set_device('gpu:0')


def run(fused, steps=6, lr=0.02, amp=True):
    paddle.seed(0)
    torch.manual_seed(0)
    model = resnet50(data_format='NHWC', num_classes=10)
    opt = paddle.optimizer.Momentum(learning_rate=lr, momentum=0.9, parameters=model.parameters(), multi_precision=True)
    if amp:
        model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16')
    orig = batchnorm.supported
    if not fused:
        batchnorm.supported = lambda *a, **k: False
    try:
        g = torch.Generator(device='cuda').manual_seed(1)
        img = paddle.to_tensor(torch.randn(8, 64, 64, 3, device='cuda', generator=g).to(torch.bfloat16 if amp else torch.float32))
        lab = paddle.to_tensor(torch.randint(0, 10, (8,), device='cuda', generator=g))
        losses, grads = [], None
        for i in range(steps):
            loss = paddle.nn.functional.cross_entropy(model(img), lab)
            loss.backward()
            if i == 0:
                grads = {n: p._t.grad.detach().float().clone() for n, p in model.named_parameters() if p._t.grad is not None}
            opt.step()
            opt.clear_grad()
            losses.append(round(float(loss), 4))
        dts = {str(p._t.dtype) for n, p in model.named_parameters() if 'bn' in n}
        return losses, grads, dts
    finally:
        batchnorm.supported = orig


import sys as _s
amp = len(_s.argv) < 2 or _s.argv[1] != 'fp32'
lf, gf, dtf = run(True, amp=amp, lr=0.002)
lu, gu, dtu = run(False, amp=amp, lr=0.002)
print('bn param dtypes', dtf, dtu)
print('fused  losses', lf)
print('unfused losses', lu)
worst = sorted(((float((gf[n] - gu[n]).norm() / (gu[n].norm() + 1e-12)), n) for n in gu if n in gf), reverse=True)[:12]
for e, n in worst:
    print(f"{e:9.4f} {n} {list(gu[n].shape)}")
