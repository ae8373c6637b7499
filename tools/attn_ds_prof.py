"""Kernel-level view of the flash backward forms on the GPT-3 1.3B attention shape (B16 S1024 H16
D128 causal, packed QKV, dropout 0.1 as in the bench): run under rocprofv3 --kernel-trace --stats.
argv[1]: 'ds' (materialised dS) or 'rc' (recompute pair)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle  # noqa: F401
    from paddle import ops
    from paddle.ops import _native
    _native._load()
    ops.flash_attn.set_ds_backward(sys.argv[1] == 'ds')
    if len(sys.argv) > 2:  # block-order group of the dS module (pair_order G)
        _native.lib.pa_flash_ds_set_pair_group(int(sys.argv[2]))
    if os.environ.get('DQ_DMA') is not None:  # dQ-from-dS kernel: 0 register-staged, 3 / 4 LDS-DMA ring depth
        _native.lib.pa_flash_ds_set_dq_dma(int(os.environ['DQ_DMA']))
    qkv = torch.randn(16, 1024, 3, 16, 128, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(16, 1024, 16, 128, device='cuda', dtype=torch.bfloat16)
    for _ in range(12):
        o = ops.flash_attn.flash_attention_packed_ex(qkv, True, dropout=0.1)
        o.backward(g)
        qkv.grad = None
    torch.cuda.synchronize()
    print('done', sys.argv[1], flush=True)


if __name__ == '__main__':
    main()
