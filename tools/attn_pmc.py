"""Flash attention fwd + bwd on the GPT-3 1.3B shape (B16 S1024 H16 D128 causal), for
rocprofv3 --pmc counter passes (tools/gpu_check29.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle  # noqa: F401
    from paddle import ops
    from paddle.ops import _native
    _native._load()
    B, S, H, D = 16, 1024, 16, 128
    q, k, v = (torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16, requires_grad=True) for _ in range(3))
    for _ in range(2):
        o = ops.flash_attn.flash_attention(q, k, v, True)
        o.backward(torch.randn_like(o))
    torch.cuda.synchronize()
    print('ok', flush=True)


if __name__ == '__main__':
    main()
