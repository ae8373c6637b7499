"""dist.to_static beyond data parallelism, as a static Program (reference
distributed/auto_parallel/api.py:2345 to_static, static/engine.py:68 Engine): 2 gloo ranks.
argv[1]:
  shard1 / shard2 / shard3 — sharding stage 1/2/3 (AdamW) over the 2 ranks, inputs Shard(0) on the
      batch axis: optimizer states (stage 1), gradients (stage 2) and parameters (stage 3,
      segment_size 1 so every unit is released and re-gathered) sharded;
  pp_1F1B / pp_FThenB — a 2-stage pipeline (SGD): parameters placed on mesh [0] / mesh [1] by
      shard_layer, accumulate_steps 4 micro-batches in the named schedule;
  engine — auto.Engine.fit over a sharded stage-2 strategy.
After 3 steps every rank's parameters (pipeline: its own stage's) must equal a single-process run
on the full batch, and the fetched losses the full-batch losses."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402


def model():
    paddle.seed(7)
    return paddle.nn.Sequential(paddle.nn.Linear(6, 12), paddle.nn.ReLU(), paddle.nn.Linear(12, 10),
                                paddle.nn.Tanh(), paddle.nn.Linear(10, 3))


def batches():
    rng = np.random.RandomState(3)
    return [(rng.randn(8, 6).astype('float32'), rng.randint(0, 3, (8,)).astype('int64')) for _ in range(3)]


def reference(opt_fn):
    net = model()
    opt = opt_fn(net)
    losses = []
    for xs, ys in batches():
        loss = paddle.nn.functional.cross_entropy(net(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        losses.append(float(loss))
        loss.backward()
        opt.step()
        opt.clear_grad()
    return net, losses


def main():
    mode = sys.argv[1]
    dist.init_parallel_env()
    rank = dist.get_rank()
    adamw = lambda n: paddle.optimizer.AdamW(0.05, parameters=n.parameters(), weight_decay=0.01)  # noqa: E731
    sgd = lambda n: paddle.optimizer.SGD(0.3, parameters=n.parameters())  # noqa: E731
    st = dist.Strategy()
    net = model()
    mesh = dist.ProcessMesh([0, 1], dim_names=['dp'])
    if mode.startswith('shard') or mode == 'engine':
        stage = 2 if mode == 'engine' else int(mode[-1])
        st.sharding.enable = True
        st.sharding.stage = stage
        st.sharding.degree = 2
        if stage == 3:
            st.sharding.segment_size = 1
        opt_fn = adamw
    else:
        sched = mode.split('_')[1]
        dist.shard_layer(net[0], dist.ProcessMesh([0], dim_names=['pp0']))
        dist.shard_layer(net[2], dist.ProcessMesh([1], dim_names=['pp1']))
        dist.shard_layer(net[4], dist.ProcessMesh([1], dim_names=['pp1']))
        st.pipeline.enable = True
        st.pipeline.accumulate_steps = 4
        st.pipeline.schedule_mode = sched
        opt_fn = sgd
    opt = opt_fn(net)
    losses = []
    if mode == 'engine':
        from paddle.distributed.auto_parallel.static.engine import Engine

        class DS(paddle.io.Dataset):
            def __init__(self):
                self.items = [(x[i], y[i]) for x, y in batches() for i in range(8)]

            def __len__(self):
                return len(self.items)

            def __getitem__(self, i):
                return self.items[i]
        eng = Engine(net, paddle.nn.CrossEntropyLoss(), opt, strategy=st)
        hist = eng.fit(DS(), batch_size=8, epochs=1, verbose=0)
        assert eng._dist_model().is_static, eng._dist_model()._static_reason
        losses = hist['loss']
    else:
        dm = dist.to_static(net, None, paddle.nn.CrossEntropyLoss(), opt, st)
        assert dm.is_static, dm._static_reason
        for xs, ys in batches():
            if mode.startswith('shard'):
                x = dist.shard_tensor(paddle.to_tensor(xs), mesh, [dist.Shard(0)])
                y = dist.shard_tensor(paddle.to_tensor(ys), mesh, [dist.Shard(0)])
            else:
                x, y = paddle.to_tensor(xs), paddle.to_tensor(ys)
            losses.append(float(dm(x, y)))
    ref, rl = reference(opt_fn)
    if mode != 'engine':  # the Engine's DistributedBatchSampler reads each rank's own half
        np.testing.assert_allclose(losses, rl, rtol=2e-5, atol=2e-6)
    if mode.startswith('shard'):
        dm.state_dict()  # stage 3: re-materialises the released parameters
    params = list(net.parameters())
    rps = list(ref.parameters())
    own = range(len(params))
    if mode.startswith('pp'):
        own = [0, 1] if rank == 0 else [2, 3, 4, 5]  # this rank's stage
    if mode == 'engine':  # the ranks read different halves; the averaged update keeps them equal
        sums = [float(p.numpy().sum()) for p in net.parameters()]
        allv = [None, None]
        torch.distributed.all_gather_object(allv, sums)
        np.testing.assert_allclose(allv[0], allv[1], rtol=1e-6)
        return print(f'rank {rank} dist static {mode} OK (losses {losses})', flush=True)
    for i in own:
        np.testing.assert_allclose(params[i].numpy(), rps[i].numpy(), rtol=2e-5, atol=2e-6, err_msg=f'param {i}')
    if mode.startswith('pp'):  # eval after training: every rank sees every stage's trained weights
        dm.eval()
        xs, ys = batches()[0]
        ev = float(dm(paddle.to_tensor(xs), paddle.to_tensor(ys)))
        want = float(paddle.nn.functional.cross_entropy(ref(paddle.to_tensor(xs)), paddle.to_tensor(ys)))
        np.testing.assert_allclose(ev, want, rtol=2e-5, atol=2e-6)
    torch.distributed.barrier()
    print(f'rank {rank} dist static {mode} OK', flush=True)


if __name__ == '__main__':
    main()
