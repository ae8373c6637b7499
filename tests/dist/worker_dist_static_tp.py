"""dist.to_static with tensor-parallel placements as a static Program: the first Linear's weight is
Shard(1) (column parallel) and the second's Shard(0) (row parallel) on a 2-rank 'mp' mesh; the
SPMD propagation runs while the step is recorded, so its reshards (the row-parallel output's
all-reduce, the replicated input's gradient all-reduce) become program nodes.  Losses and the
gathered weights must equal a single-process run on the full model, and the recorded program
must hold the collectives (no eager fallback)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402


def model():
    paddle.seed(13)
    return paddle.nn.Sequential(paddle.nn.Linear(6, 6), paddle.nn.Tanh(), paddle.nn.Linear(6, 12), paddle.nn.Tanh(),
                                paddle.nn.Linear(12, 3))


def main():
    dist.init_parallel_env()
    rank = dist.get_rank()
    mesh = dist.ProcessMesh([0, 1], dim_names=['mp'])
    rng = np.random.RandomState(0)
    batches = [(rng.randn(8, 6).astype('float32'), rng.randint(0, 3, (8,)).astype('int64')) for _ in range(3)]
    ref = model()

    net = model()
    net[2].weight = dist.shard_tensor(net[2].weight, mesh, [dist.Shard(1)])
    net[2].bias = dist.shard_tensor(net[2].bias, mesh, [dist.Shard(0)])
    net[4].weight = dist.shard_tensor(net[4].weight, mesh, [dist.Shard(0)])
    opt = paddle.optimizer.SGD(0.2, parameters=net.parameters())
    dm = dist.to_static(net, None, paddle.nn.CrossEntropyLoss(), opt, dist.Strategy())
    assert dm.is_static, dm._static_reason
    losses = [float(dm(paddle.to_tensor(xs), paddle.to_tensor(ys))) for xs, ys in batches]
    plan = next(iter(dm._progs.values()))
    # the reshards are program nodes: the row-parallel output's all-reduce and the replicated
    # activation's identity / gradient all-reduce feeding the column-parallel layer
    assert sum(1 for n in plan[0].nodes if n.kind == 'py') >= 2
    prog = dm.dist_main_program()
    assert prog is plan[0] and dm.dist_main_program('eval') is None
    assert len(prog.reshard_nodes()) >= 2
    assert len(dm.dist_startup_program().nodes) == 0
    # the serial view: no reshard collectives, the column-parallel weight at its global shape
    ser = dm.serial_main_program()
    assert ser is not None and not ser.reshard_nodes() and len(ser.nodes) > 0
    twin = ser._meta_twins[ser._const_ids[id(net[2].weight._t)]]
    assert list(twin.shape) == [6, 12], twin.shape
    assert dm.serial_main_program("predict") is None and len(dm.serial_startup_program().nodes) == 0
    # the column-parallel weight keeps its dist attribute (global shape [6, 12], Shard(1))
    mesh_, pl, gshape = prog.dist_attr(net[2].weight)
    assert list(gshape) == [6, 12] and isinstance(pl[0], dist.Shard) and pl[0].get_dim() == 1, (pl, gshape)

    ropt = paddle.optimizer.SGD(0.2, parameters=ref.parameters())
    rl = []
    for xs, ys in batches:
        loss = paddle.nn.functional.cross_entropy(ref(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        rl.append(float(loss))
        loss.backward()
        ropt.step()
        ropt.clear_grad()
    np.testing.assert_allclose(losses, rl, rtol=1e-5, atol=1e-6)
    w2 = net[2].weight._t.detach().numpy()
    np.testing.assert_allclose(w2, np.split(ref[2].weight.numpy(), 2, 1)[rank], rtol=1e-5, atol=1e-6)
    w4 = net[4].weight._t.detach().numpy()
    np.testing.assert_allclose(w4, np.split(ref[4].weight.numpy(), 2, 0)[rank], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(net[4].bias.numpy(), ref[4].bias.numpy(), rtol=1e-5, atol=1e-6)
    # the replicated first layer sees the all-reduced input gradient of the column-parallel one
    np.testing.assert_allclose(net[0].weight.numpy(), ref[0].weight.numpy(), rtol=1e-5, atol=1e-6)
    torch.distributed.barrier()
    print(f'rank {rank} dist static tp OK', flush=True)


if __name__ == '__main__':
    main()
