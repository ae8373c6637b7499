"""Which torch ops (with input shapes) the ERNIE static step still launches besides the HIP
kernels: torch.profiler over a few steps, aten::add / fill_ / copy_ / zero_ grouped by shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else 'bf16'
    sys.argv = [sys.argv[0]]
    args = bench.parse()
    torch.cuda.set_device(0)
    step, work, *_ = bench.build_ernie_static(args, 1, 0, torch.device('cuda', 0), mode == 'fp8')
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    keys = ('aten::add', 'aten::add_', 'aten::fill_', 'aten::zero_', 'aten::copy_', 'aten::zeros', 'aten::mul',
            'aten::to', 'aten::sum')
    rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key in keys]
    rows.sort(key=lambda e: -e.count)
    for e in rows[:40]:
        print(f"{e.key:14s} x{e.count:4d}  {str(e.input_shapes)[:150]}")
    print("--- stacks of the add_ calls")
    for e in prof.key_averages(group_by_stack_n=6):
        if e.key in ('aten::add_', 'aten::zero_', 'aten::fill_'):
            print(f"{e.key} x{e.count}:", " <- ".join(str(f) for f in e.stack[:6]))


if __name__ == '__main__':
    main()
