"""ERNIE-3.0-base static AMP-O2 step (bench config 5): eager Executor vs the Executor step captured
into one hipGraph (device/cuda/graphs.py TrainStepGraph), bf16 and fp8.  usage: python ernie_graph_ab.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import bench  # noqa: E402


def timed(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, float(out.item() if hasattr(out, 'item') else out)


def main():
    sys.argv = [sys.argv[0], '--steps', '20', '--warmup', '4']
    args = bench.parse()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    from paddle.device.cuda.graphs import capture_train_step
    for mode in ('bf16', 'fp8'):
        step, work, *_ = bench.build_ernie_static(args, 1, 0, dev, mode == 'fp8')
        for _ in range(4):
            step()
        ms_e, le = timed(step, 20)
        g = capture_train_step(step.core, warmup=1)
        gstep = bench._Step(step.feed, g)
        for _ in range(3):
            gstep()
        ms_g, lg = timed(gstep, 20)
        ms_e2, le2 = timed(step, 10) if os.environ.get('AB_AGAIN') else (float('nan'), float('nan'))
        print(f"ernie {mode}: eager {ms_e:.3f} ms/step (loss {le:.4f}) | hipGraph {ms_g:.3f} ms/step (loss {lg:.4f}) "
              f"| x{ms_e / ms_g:.3f}", flush=True)
        del step, g, gstep
        import gc
        gc.collect()
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
