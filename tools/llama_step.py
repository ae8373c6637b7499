"""Run the bench's Llama-2 13B layer-stack step alone (BASELINE config 4 share) for rocprofv3.

usage: python tools/llama_step.py [steps] [warmup]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    warm = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    step, work, *_ = bench.build_llama(args, 1, 0, dev)
    for _ in range(warm):
        step()
        if os.environ.get('STEP_MARKER'):
            torch.cuda._sleep(10)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
        if os.environ.get('STEP_MARKER'):
            torch.cuda._sleep(10)  # one 'spin_kernel' per step: the rocprof step boundary
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / steps * 1e3
    print(f"llama: {ms:.3f} ms/step, {work / ms * 1e3:.0f} tok/s")


if __name__ == '__main__':
    main()
