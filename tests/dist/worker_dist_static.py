"""dist.to_static as a static Program (auto-parallel static mode, reference
distributed/auto_parallel/api.py to_static -> DistModel over a distributed program): 2 gloo ranks,
inputs sharded on the batch axis (Shard(0) on a 1-D mesh), replicated parameters.  The recorded
program runs on each rank's half batch and averages the gradients over the mesh; the result must
equal a single-process run on the full batch, and the returned loss is the global-batch mean."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402


def model():
    paddle.seed(11)
    return paddle.nn.Sequential(paddle.nn.Linear(6, 12), paddle.nn.Tanh(), paddle.nn.Linear(12, 3))


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    dist.init_parallel_env()
    rank = dist.get_rank()
    mesh = dist.ProcessMesh([0, 1], dim_names=['dp'])
    rng = np.random.RandomState(0)
    batches = [(rng.randn(8, 6).astype('float32'), rng.randint(0, 3, (8,)).astype('int64')) for _ in range(4)]

    net = model()
    opt = paddle.optimizer.SGD(0.2, parameters=net.parameters())
    st = dist.Strategy()
    if k > 1:
        st.gradient_merge.enable = True
        st.gradient_merge.k_steps = k
    dm = dist.to_static(net, None, paddle.nn.CrossEntropyLoss(), opt, st)
    assert dm.is_static, dm._static_reason
    losses = []
    for xs, ys in batches:
        x = dist.shard_tensor(paddle.to_tensor(xs), mesh, [dist.Shard(0)])
        y = dist.shard_tensor(paddle.to_tensor(ys), mesh, [dist.Shard(0)])
        losses.append(float(dm(x, y)))

    ref = model()
    ropt = paddle.optimizer.SGD(0.2, parameters=ref.parameters())
    rl = []
    for i, (xs, ys) in enumerate(batches):
        loss = paddle.nn.functional.cross_entropy(ref(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        rl.append(float(loss))
        (loss / k if k > 1 else loss).backward()
        if (i + 1) % k == 0:
            ropt.step()
            ropt.clear_grad()
    np.testing.assert_allclose(losses, rl, rtol=1e-5, atol=1e-6)
    for p, q in zip(net.parameters(), ref.parameters()):
        np.testing.assert_allclose(p.numpy(), q.numpy(), rtol=1e-5, atol=1e-6)
    torch.distributed.barrier()
    print(f'rank {rank} dist static k{k} OK', flush=True)


if __name__ == '__main__':
    main()
