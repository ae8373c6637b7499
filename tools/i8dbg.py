import sys; sys.path.insert(0, '/root/repo')
import torch, paddle
from paddle.ops import int8 as I8, _native
assert _native._load() is not None
M = N = 256; K = 128
g = torch.Generator(device='cuda').manual_seed(0)
a = torch.randint(-3, 4, (M, K), device='cuda', generator=g, dtype=torch.int32).to(torch.int8)
w = torch.randint(-3, 4, (N, K), device='cuda', generator=g, dtype=torch.int32).to(torch.int8)
ex = a.float() @ w.float().t()
one_m, one_n = torch.ones(M, device='cuda'), torch.ones(N, device='cuda')
o = I8.i8_mm(a, w, one_m, one_n).float()
print('sums ok', torch.equal(o, ex), (o - ex).abs().max().item())
o = I8.i8_mm(a, w, one_m, torch.arange(N, device='cuda').float() / 64).float()
r = ex * (torch.arange(N, device='cuda').float() / 64)[None]
print('col', (o - r).abs().max().item(), (o / ex)[0, :20].tolist())
o = I8.i8_mm(a, w, torch.arange(M, device='cuda').float() / 64, one_n).float()
r = ex * (torch.arange(M, device='cuda').float() / 64)[:, None]
print('row', (o - r).abs().max().item(), (o / ex)[:20, 0].tolist())
