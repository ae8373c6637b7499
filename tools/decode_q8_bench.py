"""Decode attention over a bf16 vs an 8-bit (int8, in-kernel dequant) paged KV cache: time per call
and effective cache bandwidth (bytes of K+V read / time) for serving-sized batches."""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
import paddle  # noqa: E402,F401
from paddle.ops import decode  # noqa: E402


def run(B, Hq, Hkv, D, L, cdt, bs=64, iters=50):
    dev = 'cuda'
    nb = (L + bs - 1) // bs
    shape = (B * nb, Hkv, bs, D)
    if cdt == torch.bfloat16:
        kc = torch.randn(shape, device=dev).bfloat16()
        vc = torch.randn(shape, device=dev).bfloat16()
        kw = {}
    else:
        kc = torch.randint(-127, 128, shape, device=dev).to(cdt)
        vc = torch.randint(-127, 128, shape, device=dev).to(cdt)
        kw = dict(k_dequant=torch.full((Hkv,), 0.01, device=dev), v_dequant=torch.full((Hkv,), 0.01, device=dev))
    bt = torch.randperm(B * nb, device=dev).reshape(B, nb).int()
    q = torch.randn(B, Hq, D, device=dev).bfloat16()
    lens = torch.full((B,), L, device=dev, dtype=torch.int32)
    for _ in range(3):
        decode.decode_attention(q, kc, vc, lens, block_tables=bt, **kw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        decode.decode_attention(q, kc, vc, lens, block_tables=bt, **kw)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / iters * 1e6
    byts = 2 * B * Hkv * L * D * kc.element_size()
    return us, byts / us / 1e3


def main():
    rows = []
    for (B, Hq, Hkv, D, L) in [(32, 32, 8, 128, 4096), (64, 32, 8, 128, 8192), (16, 64, 8, 128, 16384),
                               (128, 16, 16, 64, 2048)]:
        r = {'B': B, 'Hq': Hq, 'Hkv': Hkv, 'D': D, 'L': L}
        for name, cdt in (('bf16', torch.bfloat16), ('int8', torch.int8)):
            us, gbs = min(run(B, Hq, Hkv, D, L, cdt) for _ in range(3))  # best of 3
            r[name + '_us'] = round(us, 1)
            r[name + '_GBps'] = round(gbs, 0)
        r['speedup'] = round(r['bf16_us'] / r['int8_us'], 2)
        rows.append(r)
        print(json.dumps(r), flush=True)


if __name__ == '__main__':
    main()
