"""Times the extended flash-attention paths (dropout / mask / varlen / flashmask rows) against the
plain kernel on GPT-1.3B shapes: forward alone, backward alone (fwd+bwd minus fwd), and the
bwd/fwd ratio."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import paddle  # noqa: F401,E402
from paddle import ops  # noqa: E402
from paddle.ops import _native  # noqa: E402

_native._load()
FA = ops.flash_attn


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def case(name, B, S, H, D, causal, fwd):
    qkv = torch.randn(B, S, 3, H, D, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, S, H, D, device='cuda', dtype=torch.bfloat16)
    with torch.no_grad():
        tf = timeit(lambda: fwd(qkv))
    tfb = timeit(lambda: (lambda o: o.backward(g.view(o.shape)))(fwd(qkv)))
    flops = 4 * B * H * S * S * D * (0.5 if causal else 1.0)
    tb = tfb - tf
    print(f"{name:10s} B{B} S{S} H{H} D{D} causal={int(causal)}: fwd {tf:.3f} ms ({flops / tf / 1e9:.0f} TF)  "
          f"bwd {tb:.3f} ms ({2.5 * flops / tb / 1e9:.0f} TF)  bwd/fwd {tb / tf:.2f}", flush=True)


def main():
    for (B, S, H, D, causal) in [(8, 2048, 16, 128, True), (16, 1024, 16, 128, True), (4, 4096, 32, 64, True)]:
        case('plain', B, S, H, D, causal, lambda t: FA.flash_attention_packed(t, causal))
        case('dropout.1', B, S, H, D, causal, lambda t: FA.flash_attention_packed_ex(t, causal, dropout=0.1))
        mask = torch.randn(B, 1, S, S, device='cuda').bfloat16()
        case('mask', B, S, H, D, causal, lambda t: FA.flash_attention_ex(t[:, :, 0], t[:, :, 1], t[:, :, 2], causal,
                                                                           mask=mask))
        rows = torch.randint(S // 2, S + 1, (B, 1, S), device='cuda', dtype=torch.int32)
        case('flashmask', B, S, H, D, causal,
             lambda t: FA.flash_attention_ex(t[:, :, 0], t[:, :, 1], t[:, :, 2], causal, start_rows=rows))
        lens = torch.full((B,), S, dtype=torch.int32)
        cu = torch.cat([torch.zeros(1, dtype=torch.int32), lens.cumsum(0).int()]).cuda()

        def vl(t):
            f = t.view(B * S, 3, H, D)
            return FA.flash_attention_ex(f[:, 0], f[:, 1], f[:, 2], causal, cu_seqlens_q=cu, cu_seqlens_k=cu,
                                         max_seqlen_q=S, max_seqlen_k=S)
        case('varlen', B, S, H, D, causal, vl)


if __name__ == '__main__':
    main()
