"""Fully automatic auto-parallel (strategy.auto_mode = 'full'): the rule-based planner places a
transformer encoder layer + head on a 2-rank 'mp' mesh with no user placements — q / k / v and
linear1 column parallel, out_proj and linear2 row parallel — and dist.to_static runs the planned
step as a static Program.  Losses and the gathered weights must equal single-process training."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402


class Net(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.enc = paddle.nn.TransformerEncoderLayer(16, 4, 32, dropout=0.0)
        self.head = paddle.nn.Linear(16, 3)

    def forward(self, x):
        return self.head(self.enc(x).mean(axis=1))


def model():
    paddle.seed(21)
    return Net()


def main():
    dist.init_parallel_env()
    rank = dist.get_rank()
    dist.set_mesh(dist.ProcessMesh([0, 1], dim_names=['mp']))
    rng = np.random.RandomState(1)
    batches = [(rng.randn(4, 5, 16).astype('float32'), rng.randint(0, 3, (4,)).astype('int64')) for _ in range(3)]
    ref = model()
    net = model()
    opt = paddle.optimizer.SGD(0.1, parameters=net.parameters())
    st = dist.Strategy()
    st.auto_mode = 'full'
    dm = dist.to_static(net, None, paddle.nn.CrossEntropyLoss(), opt, st)
    losses = [float(dm(paddle.to_tensor(xs), paddle.to_tensor(ys))) for xs, ys in batches]
    kinds = sorted(k for k, _ in dm.plan.patterns)
    assert kinds == ['attention', 'ffn'], dm.plan.patterns
    assert dm.is_static, dm._static_reason
    assert dist.auto_parallel.is_dist_tensor(net.enc.self_attn.q_proj.weight)

    ropt = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
    rl = []
    for xs, ys in batches:
        loss = paddle.nn.functional.cross_entropy(ref(paddle.to_tensor(xs)), paddle.to_tensor(ys))
        rl.append(float(loss))
        loss.backward()
        ropt.step()
        ropt.clear_grad()
    np.testing.assert_allclose(losses, rl, rtol=1e-5, atol=1e-6)
    q = net.enc.self_attn.q_proj.weight._t.detach().numpy()
    np.testing.assert_allclose(q, np.split(ref.enc.self_attn.q_proj.weight.numpy(), 2, 1)[rank], rtol=1e-5, atol=1e-6)
    o = net.enc.self_attn.out_proj.weight._t.detach().numpy()
    np.testing.assert_allclose(o, np.split(ref.enc.self_attn.out_proj.weight.numpy(), 2, 0)[rank], rtol=1e-5,
                               atol=1e-6)
    np.testing.assert_allclose(net.head.weight.numpy(), ref.head.weight.numpy(), rtol=1e-5, atol=1e-6)
    torch.distributed.barrier()
    print(f'rank {rank} dist auto plan OK', flush=True)


if __name__ == '__main__':
    main()
