"""Multi-process worker: DataParallel and group-sharded stage 1/2/3 must match single-process training.

Run with torch.distributed.run (gloo, world 2). Each rank trains on its half of the global batch;
the reference (computed on every rank, no communication) trains on the full batch.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.nn as nn  # noqa: E402


class Net(nn.Layer):
    def __init__(self):
        super().__init__()
        self.emb = nn.Embedding(50, 16)
        self.blocks = nn.LayerList([nn.Sequential(nn.Linear(16, 32), nn.GELU(), nn.Linear(32, 16)) for _ in range(3)])
        self.norm = nn.LayerNorm(16)
        self.head = nn.Linear(16, 5)

    def forward(self, ids):
        h = self.emb(ids).mean(axis=1)
        for b in self.blocks:
            h = h + b(h)
        return self.head(self.norm(h))


def make(seed=7):
    paddle.seed(seed)
    return Net()


def data(step):
    g = torch.Generator().manual_seed(100 + step)
    ids = torch.randint(0, 50, (8, 6), generator=g)
    y = torch.randint(0, 5, (8,), generator=g)
    return paddle.to_tensor(ids), paddle.to_tensor(y)


def train(model, opt, rank, world, steps=4, split=True):
    losses = []
    for s in range(steps):
        ids, y = data(s)
        if split:
            n = ids.shape[0] // world
            ids, y = ids[rank * n:(rank + 1) * n], y[rank * n:(rank + 1) * n]
        loss = paddle.nn.functional.cross_entropy(model(ids), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    return losses


def params_of(model):
    inner = model._layers if hasattr(model, '_layers') else model
    sd = model.state_dict() if hasattr(model, '_engine') or '_engine' in model.__dict__ else inner.state_dict()
    return {k: v.numpy().astype(np.float64) for k, v in sd.items()}


def make_opt(kind, params):
    clip = nn.ClipGradByGlobalNorm(0.5)
    if kind == 'momentum':  # sharded Momentum (velocity sharded like the Adam moments), L2 decay, Nesterov
        return paddle.optimizer.Momentum(learning_rate=0.05, momentum=0.9, parameters=params, use_nesterov=True,
                                         weight_decay=1e-3, grad_clip=clip)
    if kind == 'sgd':
        return paddle.optimizer.SGD(learning_rate=0.1, parameters=params, weight_decay=1e-3, grad_clip=clip)
    return paddle.optimizer.AdamW(learning_rate=0.01, parameters=params, grad_clip=clip)


def main():
    mode = sys.argv[1]
    kind = sys.argv[2] if len(sys.argv) > 2 else 'adamw'
    dist.init_parallel_env()
    rank, world = dist.get_rank(), dist.get_world_size()
    ref = make()
    ropt = make_opt(kind, ref.parameters())
    train(ref, ropt, rank, world, split=False)

    model = make()
    opt = make_opt(kind, model.parameters())
    if mode == 'dp':
        model = paddle.DataParallel(model)
    elif mode == 'p_g_os_keep':  # stage 3 without the backward re-gather (reshard_after_forward=False)
        model, opt, _ = dist.sharding.group_sharded_parallel(model, opt, level='p_g_os', segment_size=64,
                                                             reshard_after_forward=False)
        assert not model._engine.reshard_after_forward
    elif mode.endswith('_offload'):  # optimizer state in host memory, host-runtime update
        level = mode[:-len('_offload')]
        model, opt, _ = dist.sharding.group_sharded_parallel(model, opt, level=level, segment_size=64, offload=True)
        eng = model._engine
        assert eng.offload and all(not a['m'].is_cuda and not a['master'].is_cuda for a in eng.arenas.values())
        mode = level
    else:
        model, opt, _ = dist.sharding.group_sharded_parallel(model, opt, level=mode, segment_size=64)
        if mode == 'p_g_os':
            assert model._engine.reshard_after_forward  # CPU default
    train(model, opt, rank, world, split=True)
    want = params_of(ref)
    if mode in ('os', 'os_g'):
        # read through the ORIGINAL layer right after the last step: the stage-1/2 parameter
        # all-gathers are asynchronous and must be waited for by the inner state_dict
        inner = {k: v.numpy().astype(np.float64) for k, v in model._layers.state_dict().items()}
        for k in want:
            err = np.abs(inner[k] - want[k]).max()
            assert err < 2e-5, ('inner', mode, kind, k, err)
    got = params_of(model)
    for k in want:
        err = np.abs(got[k] - want[k]).max()
        assert err < 2e-5, (mode, kind, k, err)
    print(f"rank{rank} {sys.argv[1]} OK", flush=True)


if __name__ == '__main__':
    main()
