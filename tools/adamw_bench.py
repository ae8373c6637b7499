"""Fused AdamW streaming update (csrc/embed_rope_optim.hip) on a GPT-3 1.3B-sized flat buffer:
fp32 master/m/v, bf16 grad and model copy (28 B/param).  A/B of nontemporal accesses and
blocks per CU; prints us and achieved HBM TB/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import paddle  # noqa: F401
    from paddle.ops import _native, optim
    _native._load()
    n = 1_316_000_000
    dev = 'cuda'
    master = torch.randn(n, device=dev)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    g = torch.randn(n, device=dev, dtype=torch.bfloat16)
    low = master.bfloat16()

    def run():
        optim.adamw_flat(master, g, m, v, low, 1e-4, 0.9, 0.95, 1e-8, 0.01, 0.9, 0.95)

    for nt in (0, 1):
        for bpc in (0, 4, 8, 16):
            _native.lib.pa_adamw_tune(nt, bpc)
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) / 1e3 / 5
            print(f"nontemporal={nt} blocks/CU={bpc or 'one-shot'}: {t*1e6:8.1f} us  {28 * n / t / 1e12:5.2f} TB/s", flush=True)
    _native.lib.pa_adamw_tune(0, 0)


if __name__ == '__main__':
    main()
