"""Kernel census of the masked vs plain head_dim-64 flash forward + backward (ERNIE shape), for
rocprofv3 --kernel-trace --stats."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import paddle  # noqa: E402,F401
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

FA = ops.flash_attn


def main():
    _native._load()
    B, S, H, D = 64, 512, 12, 64
    q, k, v = (torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    allk = torch.ones(B, 1, 1, S, dtype=torch.bool, device='cuda')
    g = torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16)
    for _ in range(5):
        FA.flash_attention_ex(q, k, v, mask=allk, dropout=0.1).backward(g)   # EXT 7
        FA.flash_attention_ex(q, k, v, mask=allk).backward(g)                # EXT 3
        FA.flash_attention_ex(q, k, v, dropout=0.1).backward(g)              # EXT 5
        FA.flash_attention(q, k, v, False).backward(g)                       # plain
    torch.cuda.synchronize()
    print('ok')


if __name__ == '__main__':
    main()
