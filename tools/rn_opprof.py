"""torch.profiler attribution of the ResNet50 bench step's non-HIP device work: which Python call
sites launch the aten elementwise kernels (adds, fills, copies) left in the step."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import bench
    args = types.SimpleNamespace(resnet_batch=int(os.environ.get('RN_BATCH', '256')), resnet_model='resnet50')
    dev = torch.device('cuda', 0)
    import paddle
    paddle.set_device('gpu:0')
    step, *_ = bench.build_resnet(args, 1, 0, dev)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as p:
        step()
        torch.cuda.synchronize()
    ka = p.key_averages(group_by_input_shape=True, group_by_stack_n=6)
    rows = [e for e in ka if e.key.startswith('aten::') and e.device_time_total > 0 and
            not e.key.startswith(('aten::empty', 'aten::to', 'aten::_to'))]
    rows.sort(key=lambda e: -e.device_time_total)
    for e in rows[:25]:
        print(f"{e.device_time_total/1e3:8.3f} ms  n={e.count:4d}  {e.key}  shapes={str(e.input_shapes)[:120]}")
        for fr in e.stack[:6]:
            print('        ', fr)
    print(p.key_averages().table(sort_by='device_time_total', row_limit=30, max_name_column_width=90))


if __name__ == '__main__':
    main()
