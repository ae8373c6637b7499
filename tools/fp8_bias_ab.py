"""Same-process A/B on the bench's ERNIE fp8 static step: fp8 Linear / FFN bias gradients from
the dY cast's column sums (ops.fp8.BIAS_FROM_CAST = True) vs a separate column-sum pass."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    sys.argv = [sys.argv[0]]
    import bench
    import paddle  # noqa: F401
    from paddle.ops import fp8
    args = bench.parse()
    torch.cuda.set_device(0)
    step, *_ = bench.build_ernie_static(args, 1, 0, torch.device('cuda', 0), True)
    for _ in range(3):
        step()
    res = {True: [], False: []}
    for _ in range(4):
        for s in (True, False):
            fp8.BIAS_FROM_CAST = s
            step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                step()
            e1.record()
            torch.cuda.synchronize()
            res[s].append(e0.elapsed_time(e1) / 10)
    fp8.BIAS_FROM_CAST = True
    for s in (True, False):
        print(f"ernie fp8 bias grads from the dY cast={s}: median {statistics.median(res[s]):.3f} ms/step  "
              f"min {min(res[s]):.3f}", flush=True)


if __name__ == '__main__':
    main()
