"""Static Program + Executor tensor parallelism over gloo ranks (reference: fleet static mode with
the mpu layers, whose c_identity / c_allreduce_sum / c_concat ops sit in the program).
argv[1]: 'tp' (mp degree = world) or 'tpdp' (mp 2 x dp 2 on 4 ranks).  Each rank records
x -> ColumnParallelLinear -> relu -> RowParallelLinear -> ParallelCrossEntropy over a
vocab-parallel head, trains with SGD through fleet.distributed_optimizer, and must end with the
shards of a single-process run on the full weights / full batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.static as static  # noqa: E402
from paddle.distributed import fleet  # noqa: E402


def gather(t, group):
    parts = [torch.empty_like(t) for _ in range(group.nranks)]
    tdist.all_gather(parts, t.contiguous(), group=group.pg)
    return parts


def main():
    mode = sys.argv[1]
    world = int(os.environ['WORLD_SIZE'])
    mp = 2
    dp = world // mp
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': dp, 'mp_degree': mp, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    rank = dist.get_rank()
    mpg = hcg.get_model_parallel_group()
    dp_rank = hcg.get_data_parallel_rank()
    mpu = fleet.meta_parallel
    paddle.seed(7)
    paddle.enable_static()
    main_p, startup = static.Program(), static.Program()
    with static.program_guard(main_p, startup):
        x = static.data('x', [None, 6], 'float32')
        y = static.data('y', [None, 1], 'int64')
        l1 = mpu.ColumnParallelLinear(6, 8, has_bias=True, gather_output=False)
        l2 = mpu.RowParallelLinear(8, 10, has_bias=True, input_is_parallel=True)
        head = mpu.ColumnParallelLinear(10, 6, has_bias=False, gather_output=False)
        h = paddle.nn.functional.relu(l1(x))
        logits = head(l2(h))
        loss = mpu.ParallelCrossEntropy()(logits, y).mean()
        opt = fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.3))
        opt.minimize(loss)
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    # full initial weights (column shards of l1 / head, row shards of l2) for the reference
    W1 = torch.cat(gather(l1.weight._t.detach(), mpg), 1)
    b1 = torch.cat(gather(l1.bias._t.detach(), mpg), 0)
    W2 = torch.cat(gather(l2.weight._t.detach(), mpg), 0)
    b2 = l2.bias._t.detach().clone()
    W3 = torch.cat(gather(head.weight._t.detach(), mpg), 1)
    rng = np.random.RandomState(0)
    batches = [(rng.randn(8, 6).astype('float32'), rng.randint(0, 6, (8, 1)).astype('int64')) for _ in range(3)]
    half = 8 // dp
    for xs, ys in batches:
        exe.run(main_p, feed={'x': xs[dp_rank * half:(dp_rank + 1) * half],
                              'y': ys[dp_rank * half:(dp_rank + 1) * half]}, fetch_list=[loss])
    # reference: full model, full batch, plain SGD
    ps = [t.clone().requires_grad_() for t in (W1, b1, W2, b2, W3)]
    for xs, ys in batches:
        xt, yt = torch.from_numpy(xs), torch.from_numpy(ys).view(-1)
        lg = (torch.relu(xt @ ps[0] + ps[1]) @ ps[2] + ps[3]) @ ps[4]
        ls = torch.nn.functional.cross_entropy(lg, yt)
        for p in ps:
            p.grad = None
        ls.backward()
        with torch.no_grad():
            for p in ps:
                p -= 0.3 * p.grad
    r = hcg.get_model_parallel_rank()
    c1, c3 = W1.shape[1] // mp, W3.shape[1] // mp
    rows2 = W2.shape[0] // mp
    ref = {'w1': ps[0][:, r * c1:(r + 1) * c1], 'b1': ps[1][r * c1:(r + 1) * c1],
           'w2': ps[2][r * rows2:(r + 1) * rows2], 'b2': ps[3], 'w3': ps[4][:, r * c3:(r + 1) * c3]}
    got = {'w1': l1.weight._t, 'b1': l1.bias._t, 'w2': l2.weight._t, 'b2': l2.bias._t, 'w3': head.weight._t}
    for k in ref:
        np.testing.assert_allclose(got[k].detach().numpy(), ref[k].detach().numpy(), rtol=1e-4, atol=1e-5,
                                   err_msg=k)
    print(f"rank{rank} static {mode} OK", flush=True)


if __name__ == '__main__':
    main()
