"""Static Program + Executor data parallelism over 2 gloo ranks (reference: fleet collective
static mode, raw_program_optimizer.py c_broadcast / c_allreduce_sum): each rank builds the program
from a DIFFERENT seed and feeds half of every batch; after the parameter broadcast and gradient
averaging the weights match a single-process run on the full batch.
argv[1]: 'fleet' (fleet.distributed_optimizer), 'fleet_merge' (+ strategy gradient merge k=2),
'pass' (paddle.distributed.passes auto_parallel_data_parallel_optimization)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.static as static  # noqa: E402
from paddle.distributed import fleet  # noqa: E402


def build(seed, opt_fn):
    paddle.seed(seed)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 6], 'float32')
        y = static.data('y', [None, 1], 'int64')
        h = static.nn.fc(x, 12, activation='relu')
        logits = static.nn.fc(h, 3)
        loss = paddle.nn.functional.cross_entropy(logits, y)
        opt_fn().minimize(loss)
    return main, startup, loss


def main():
    mode = sys.argv[1]
    s = fleet.DistributedStrategy()
    k = 1
    if mode == 'fleet_merge':
        s.gradient_merge = True
        s.gradient_merge_configs = {'k_steps': 2, 'avg': True}
        k = 2
    fleet.init(is_collective=True, strategy=s)
    rank, world = dist.get_rank(), dist.get_world_size()
    paddle.enable_static()
    mom = lambda: paddle.optimizer.Momentum(learning_rate=0.2, momentum=0.9)  # noqa: E731
    if mode == 'pass':
        main_p, startup, loss = build(100 + rank, mom)
        from paddle.distributed.passes import new_pass
        new_pass('auto_parallel_data_parallel_optimization', {'fuse_grad_size_in_MB': 0.0005}).apply(
            [main_p], [startup])
    else:
        main_p, startup, loss = build(100 + rank, lambda: fleet.distributed_optimizer(mom()))
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    rng = np.random.RandomState(0)
    batches = []
    for _ in range(3 * k):
        xs = rng.randn(16, 6).astype('float32')
        batches.append((xs, (xs[:, :3].argmax(1)).reshape(-1, 1).astype('int64')))
    half = 16 // world
    for xs, ys in batches:
        exe.run(main_p, feed={'x': xs[rank * half:(rank + 1) * half], 'y': ys[rank * half:(rank + 1) * half]},
                fetch_list=[loss])
    got = [p.numpy().copy() for p in main_p.all_parameters()]
    # single-process reference: rank 0's initial weights, the full batch (k micro-batches merged)
    ref_main, ref_startup, ref_loss = build(100, mom)
    exe.run(ref_startup)
    for i in range(0, len(batches), k):
        xs = np.concatenate([b[0] for b in batches[i:i + k]])
        ys = np.concatenate([b[1] for b in batches[i:i + k]])
        exe.run(ref_main, feed={'x': xs, 'y': ys}, fetch_list=[ref_loss])
    for a, b in zip(got, [p.numpy() for p in ref_main.all_parameters()]):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5)
    print(f"rank{rank} static dp {mode} OK", flush=True)


if __name__ == '__main__':
    main()
