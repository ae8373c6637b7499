"""Per-step GPU time of the bench's GPT-3 1.3B step (events around every step, no host syncs
inside the loop) after W warmup steps: shows how many steps the throughput takes to settle."""
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch


def main():
    import bench
    W = int(os.environ.get('W', '3'))
    n = int(os.environ.get('N', '30'))
    args = types.SimpleNamespace(model='gpt3-1.3b', micro_batch=16, seq=1024, sharding='p_g_os', dropout=0.1,
                                 attn_dropout=0.1, graph=False, warmup=W)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(0)
    import paddle
    paddle.seed(1234)
    step, *_ = bench.build_gpt(args, 1, 0, dev)
    for _ in range(W):
        step()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    ev[0].record()
    for i in range(n):
        step()
        ev[i + 1].record()
    torch.cuda.synchronize()
    ts = [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]
    print('per-step ms:', ' '.join(f'{t:.1f}' for t in ts))
    print(f'first 10 mean {sum(ts[:10]) / 10:.2f}  last 10 mean {sum(ts[-10:]) / 10:.2f}')
    print('memory reserved GB', torch.cuda.memory_reserved() / 1e9, 'allocated', torch.cuda.memory_allocated() / 1e9)


if __name__ == '__main__':
    main()
