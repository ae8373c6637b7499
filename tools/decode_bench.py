"""Decode attention (csrc/decode_attn.hip) bandwidth on Llama-2-13B-shaped layers (40 heads x 128,
MHA) and a GQA shape: KV bytes read per step / time, contiguous and paged caches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def bench(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 1e3 / n


def main():
    import paddle  # noqa: F401
    from paddle.ops import decode
    dev, bf = 'cuda', torch.bfloat16
    for (Hq, Hkv, D) in [(40, 40, 128), (32, 8, 128)]:
        for B in (16, 32, 64):
            for L in (2048, 4096):
                kc = torch.randn(B, Hkv, L, D, device=dev, dtype=bf)
                vc = torch.randn_like(kc)
                q = torch.randn(B, Hq, D, device=dev, dtype=bf)
                lens = torch.full((B,), L, device=dev, dtype=torch.int32)
                t = bench(lambda: decode.decode_attention(q, kc, vc, lens))
                byt = 2 * kc.numel() * 2
                bs = 64
                nblk = B * L // bs
                kp = kc.reshape(B, Hkv, L // bs, bs, D).permute(0, 2, 1, 3, 4).reshape(nblk, Hkv, bs, D).contiguous()
                vp = vc.reshape(B, Hkv, L // bs, bs, D).permute(0, 2, 1, 3, 4).reshape(nblk, Hkv, bs, D).contiguous()
                bt = torch.arange(nblk, device=dev, dtype=torch.int32).reshape(B, L // bs)
                tp = bench(lambda: decode.decode_attention(q, kp, vp, lens, block_tables=bt))
                print(f"Hq{Hq} Hkv{Hkv} D{D} B{B:3d} L{L}: contiguous {t*1e6:8.1f} us {byt/t/1e12:5.2f} TB/s | "
                      f"paged(bs64) {tp*1e6:8.1f} us {byt/tp/1e12:5.2f} TB/s", flush=True)
                del kc, vc, kp, vp


if __name__ == '__main__':
    main()
