import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import paddle  # noqa
from paddle.ops import batchnorm
for dt in (torch.float32, torch.bfloat16):
    for shape in [(2, 5, 5, 96), (2, 5, 5, 64), (1, 3, 4, 48), (4, 6, 6, 96)]:
        C = shape[-1]
        torch.manual_seed(0)
        x = (torch.randn(*shape, device='cuda') * 2 + 3).to(dt)
        g = torch.ones(C, device='cuda'); b = torch.zeros(C, device='cuda')
        rm, rv = torch.zeros(C, device='cuda'), torch.ones(C, device='cuda')
        y = batchnorm.bn_act_nhwc(x, g, b, rm, rv, 1e-5, 0.9, True, False, None).float().reshape(-1, C)
        xr = x.float().reshape(-1, C)
        yr = (xr - xr.mean(0)) / torch.sqrt(xr.var(0, unbiased=False) + 1e-5)
        err = (y - yr).abs()
        bad = (err > 0.05).nonzero()
        print(dt, shape, 'maxerr', err.max().item(), 'bad rows', sorted(set(bad[:, 0].tolist()))[:20], 'bad cols', sorted(set(bad[:, 1].tolist()))[:40], flush=True)
        print('  mean err', (rm / 0.1 - xr.mean(0)).abs().max().item(), flush=True)
