"""A/B of the column-sum kernels' row order (pa_act_cs_set_interleave: 1 round-robin groups of 4
rows over the row blocks, 0 contiguous per-block chunks) on the bench's ERNIE bf16 / fp8 static
steps and the GPT-3 1.3B step: interleaved rounds in one process, ms/step per setting.
usage: python tools/cs_order_ab.py [ernie_bf16,ernie_fp8,gpt]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    which = (sys.argv[1] if len(sys.argv) > 1 else 'ernie_bf16,ernie_fp8,gpt').split(',')
    sys.argv = [sys.argv[0]]
    import bench
    import paddle  # noqa: F401
    from paddle.ops import _native
    L = _native._load()
    args = bench.parse()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    for name in which:
        if name == 'gpt':
            step, *_ = bench.build_gpt(args, 1, 0, dev)
        else:
            step, *_ = bench.build_ernie_static(args, 1, 0, dev, name == 'ernie_fp8')
        for _ in range(3):
            step()
        res = {1: [], 0: []}
        reps = 3 if name == 'gpt' else 10
        for _ in range(4):
            for s in (1, 0):
                L.pa_act_cs_set_interleave(s)
                step()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    step()
                e1.record()
                torch.cuda.synchronize()
                res[s].append(e0.elapsed_time(e1) / reps)
        L.pa_act_cs_set_interleave(1)
        for s in (1, 0):
            print(f"{name}: column-sum row order interleave={s}: median {statistics.median(res[s]):.3f} ms/step  "
                  f"min {min(res[s]):.3f}", flush=True)
        del step
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
