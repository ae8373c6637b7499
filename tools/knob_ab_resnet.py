"""Same-process A/B of an int knob of the kernel library on the ResNet50 bench step (interleaved
rounds, ms/step per setting). KNOB: the setter (default pa_bn_set_interleave: 1 round-robin row
groups, 0 contiguous per-block chunks); VALUES: comma list (default 1,0)."""
import os
import statistics
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import bench
    import paddle
    from paddle.ops import _native
    L = _native._load()
    paddle.set_device('gpu:0')
    step, *_ = bench.build_resnet(types.SimpleNamespace(resnet_batch=256, resnet_model='resnet50', steps=10, warmup=3), 1, 0, torch.device('cuda', 0))
    for _ in range(3):
        step()
    knob = getattr(L, os.environ.get('KNOB', 'pa_bn_set_interleave'))
    settings = [int(v) for v in os.environ.get('VALUES', '1,0').split(',')]
    res = {s: [] for s in settings}
    for _ in range(4):
        for s in settings:
            knob(s)
            step()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                step()
            e1.record()
            torch.cuda.synchronize()
            res[s].append(e0.elapsed_time(e1) / 5)
    for s in settings:
        print(f"{os.environ.get('KNOB', 'pa_bn_set_interleave')}={s}: median {statistics.median(res[s]):.3f} ms/step  min {min(res[s]):.3f}",
              flush=True)


if __name__ == '__main__':
    main()
