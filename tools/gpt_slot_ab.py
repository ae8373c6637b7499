"""Same-process A/B of GPT-3 1.3B (bench config) with the norm-parameter gradient slot
accumulation on vs off (ops.conv.SLOT_ACCUM, ops.batchnorm.SLOT_ACCUM), alternating blocks."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    torch.cuda.set_device(0)
    step, work, *_ = bench.build_gpt(args, 1, 0, torch.device("cuda", 0))
    from paddle.ops import fused as C, batchnorm as BN
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    res = {True: [], False: []}
    for rep in range(3):
        for on in (True, False):
            C.SLOT_ACCUM = BN.SLOT_ACCUM = on
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            res[on].append((time.perf_counter() - t0) / 5 * 1e3)
    for on in (True, False):
        print(f"slot accumulation {'on ' if on else 'off'}: " + " ".join(f"{m:.2f}" for m in res[on]) +
              f" ms/step -> {work / (min(res[on]) / 1e3):.0f} tok/s best")


if __name__ == '__main__':
    main()
