"""Auto-parallel optimizer sharding (shard_optimizer + ShardingStage1/2/3, DistModel Strategy with
sharding / gradient merge / recompute, shard_scaler) on a 2-rank gloo mesh must match
single-process training on the full batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402


class MLP(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.l1 = paddle.nn.Linear(8, 16)
        self.l2 = paddle.nn.Linear(16, 4)

    def forward(self, x):
        return self.l2(paddle.nn.functional.relu(self.l1(x)))


def data(step, world):
    g = torch.Generator().manual_seed(100 + step)
    x = torch.randn(4 * world, 8, generator=g)
    y = torch.randint(0, 4, (4 * world,), generator=g)
    return x, y


def reference(steps, world, k=1):
    paddle.seed(5)
    m = MLP()
    opt = paddle.optimizer.AdamW(1e-2, parameters=m.parameters())
    for s in range(steps):
        x, y = data(s, world)
        loss = paddle.nn.functional.cross_entropy(m(paddle.to_tensor(x)), paddle.to_tensor(y))
        (loss / k).backward()
        if (s + 1) % k == 0:
            opt.step()
            opt.clear_grad()
    return {n: p.numpy() for n, p in m.named_parameters()}


def run(mode, steps, world, rank):
    mesh = dist.ProcessMesh(list(range(world)), dim_names=['dp'])
    paddle.seed(5)
    m = MLP()
    opt = paddle.optimizer.AdamW(1e-2, parameters=m.parameters())
    k = 1
    if mode == 'plain':
        opt = dist.shard_optimizer(opt)
    elif mode in ('stage1', 'stage2'):
        stage = dist.ShardingStage1(mesh) if mode == 'stage1' else dist.ShardingStage2(mesh)
        opt = dist.shard_optimizer(opt, stage)
        assert opt._engine is not None and opt._engine.world == world
    loss_fn = paddle.nn.CrossEntropyLoss()
    if mode == 'distmodel':
        k = 2
        st = dist.Strategy({'sharding': {'enable': True, 'stage': 3},
                            'gradient_merge': {'enable': True, 'k_steps': k, 'avg': True},
                            'recompute': {'enable': True}})
        dm = dist.to_static(m, None, loss_fn, opt, strategy=st)
        assert dm._opt._engine is not None and dm._opt._engine.level == 3
        dm.train()
    for s in range(steps):
        x, y = data(s, world)
        xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
        if mode == 'distmodel':
            dm(paddle.to_tensor(xs), paddle.to_tensor(ys))
            continue
        loss = loss_fn(m(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        loss.backward()
        opt.step()
        opt.clear_grad()
    ref = reference(steps, world, k)
    if mode == 'distmodel':
        got = {n: v.numpy() for n, v in dm._opt._engine.model.state_dict().items()} if False else None
        from paddle.parallel.sharding import gathered_state_dict
        got = {n: v.numpy() for n, v in gathered_state_dict(m, dm._opt._engine).items()}
    else:
        got = {n: p.numpy() for n, p in m.named_parameters()}
    for n, v in ref.items():
        err = float(np.abs(got[n] - v).max())
        assert err < 2e-5, (mode, n, err)
    # shard_scaler: ranks agree on found_inf even when only one rank overflows
    sc = dist.shard_scaler(paddle.amp.GradScaler(init_loss_scaling=8.0))
    found = torch.tensor(1.0 if rank == 0 else 0.0)
    assert sc._sync_found_inf(found) is True
    print(f"rank{rank} auto_shard {mode} OK", flush=True)


if __name__ == '__main__':
    dist.init_parallel_env()
    run(sys.argv[1], 4, dist.get_world_size(), dist.get_rank())
    # orderly teardown: a rank that exits while gloo's pair threads still run aborts at exit
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
