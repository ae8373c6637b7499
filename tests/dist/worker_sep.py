"""Segment parallel (``sep`` axis) workers: sep alone and combined with mp / dp / sharding must train
exactly like one process on the whole batch (reference test/collective/fleet/hybrid_parallel_sep_model.py).

Each rank takes its data-parallel slice of the global batch (dp x sharding ranks see different
samples), splits every sequence over its sep peers, runs the net on its segment and gathers the
logits over sep (all-gather forward, own-slice backward), so each sep rank's gradient is a partial
sum that the framework must add up over sep (and average over dp)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
from paddle.autograd import PyLayer  # noqa: E402
from paddle.distributed import fleet  # noqa: E402

V, H, F, S, B = 16, 8, 12, 8, 2  # vocab, hidden, ffn, seq, per-replica batch


class SepConcat(PyLayer):
    @staticmethod
    def forward(ctx, x, axis, group):
        parts = []
        dist.all_gather(parts, x, group=group)
        ctx.axis, ctx.group = axis, group
        with paddle.no_grad():
            return paddle.concat(parts, axis=axis)

    @staticmethod
    def backward(ctx, g):
        n = dist.get_world_size(ctx.group)
        return paddle.split(g, n, axis=ctx.axis)[dist.get_rank(ctx.group)]


def sep_split(x, axis, group):
    n = dist.get_world_size(group)
    return paddle.split(x, n, axis=axis)[dist.get_rank(group)]


def full_weights():
    rs = np.random.RandomState(7)
    return {'emb': rs.randn(V, H).astype('float32') * 0.5, 'w1': rs.randn(H, F).astype('float32') * 0.3,
            'b1': rs.randn(F).astype('float32') * 0.1, 'w2': rs.randn(F, H).astype('float32') * 0.3,
            'b2': rs.randn(H).astype('float32') * 0.1}


class Net(paddle.nn.Layer):
    def __init__(self, mp, sep_group=None):
        super().__init__()
        W = full_weights()
        self.sep_group = sep_group
        self.emb = paddle.nn.Embedding(V, H)
        self.emb.weight.set_value(W['emb'])
        if mp > 1:
            hcg = fleet.get_hybrid_communicate_group()
            r = hcg.get_model_parallel_rank()
            self.fc1 = fleet.meta_parallel.ColumnParallelLinear(H, F, gather_output=False)
            self.fc2 = fleet.meta_parallel.RowParallelLinear(F, H, input_is_parallel=True)
            self.fc1.weight.set_value(np.split(W['w1'], mp, 1)[r])
            self.fc1.bias.set_value(np.split(W['b1'], mp, 0)[r])
            self.fc2.weight.set_value(np.split(W['w2'], mp, 0)[r])
        else:
            self.fc1 = paddle.nn.Linear(H, F)
            self.fc2 = paddle.nn.Linear(F, H)
            self.fc1.weight.set_value(W['w1'])
            self.fc1.bias.set_value(W['b1'])
            self.fc2.weight.set_value(W['w2'])
        self.fc2.bias.set_value(W['b2'])

    def forward(self, ids, labels):
        if self.sep_group is not None:
            ids = sep_split(ids, 1, self.sep_group)
        h = self.emb(ids)
        h = h + self.fc2(paddle.nn.functional.gelu(self.fc1(h)))
        logits = paddle.matmul(h, self.emb.weight, transpose_y=True)
        if self.sep_group is not None:
            logits = SepConcat.apply(logits, 1, self.sep_group)
        return paddle.nn.functional.cross_entropy(logits.reshape([-1, V]), labels.reshape([-1])).mean()


def batches(n_rep, steps=3):
    rs = np.random.RandomState(11)
    return [(rs.randint(0, V, (B * n_rep, S)), rs.randint(0, V, (B * n_rep, S))) for _ in range(steps)]


def main(mode):
    deg = {'sep': dict(sep=2), 'sepmp': dict(sep=2, mp=2), 'sepdp': dict(sep=2, dp=2),
           'sepsh': dict(sep=2, sh=2), 'sep4': dict(sep=4)}[mode]
    sep, mp, dp, sh = deg.get('sep', 1), deg.get('mp', 1), deg.get('dp', 1), deg.get('sh', 1)
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': dp, 'mp_degree': mp, 'pp_degree': 1, 'sharding_degree': sh,
                        'sep_degree': sep}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    assert hcg.get_sep_parallel_world_size() == sep
    assert hcg.get_dp_sep_parallel_group() is not None
    # the reference's precedence: mp wins over sep, sep over sharding
    want = fleet.ParallelMode.TENSOR_PARALLEL if mp > 1 else fleet.ParallelMode.SEGMENT_PARALLEL
    assert hcg.get_parallel_mode() == want, (hcg.get_parallel_mode(), want)

    paddle.seed(100 + dist.get_rank())  # deliberately different init: broadcast must fix it
    model = Net(mp, hcg.get_sep_parallel_group())
    model = fleet.distributed_model(model)
    opt = paddle.optimizer.SGD(learning_rate=0.5, parameters=model.parameters())
    opt = fleet.distributed_optimizer(opt)

    n_rep = dp * sh
    rep = hcg.get_data_parallel_rank() * sh + hcg.get_sharding_parallel_rank()
    data = batches(n_rep)
    losses = []
    for ids, lab in data:
        sl = slice(rep * B, (rep + 1) * B)
        loss = model(paddle.to_tensor(ids[sl]), paddle.to_tensor(lab[sl]))
        loss.backward()
        opt.step()
        opt.clear_grad()
        t = loss._t.detach().clone().reshape(1)
        torch.distributed.all_reduce(t)  # mean over replicas = the global-batch loss
        losses.append(float(t) / dist.get_world_size() * 1.0)

    # single-process reference on the whole global batch
    ref = Net(1, None)
    ropt = paddle.optimizer.SGD(learning_rate=0.5, parameters=ref.parameters())
    rlosses = []
    for ids, lab in data:
        l2 = ref(paddle.to_tensor(ids), paddle.to_tensor(lab))
        l2.backward()
        ropt.step()
        ropt.clear_grad()
        rlosses.append(float(l2))
    np.testing.assert_allclose(losses, rlosses, rtol=1e-5, atol=1e-6)
    inner = model._layers if hasattr(model, '_layers') else model
    np.testing.assert_allclose(inner.emb.weight.numpy(), ref.emb.weight.numpy(), rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(inner.fc2.bias.numpy(), ref.fc2.bias.numpy(), rtol=1e-5, atol=1e-6)
    if mp > 1:
        r = hcg.get_model_parallel_rank()
        np.testing.assert_allclose(inner.fc1.weight.numpy(), np.split(ref.fc1.weight.numpy(), mp, 1)[r],
                                   rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(inner.fc2.weight.numpy(), np.split(ref.fc2.weight.numpy(), mp, 0)[r],
                                   rtol=1e-5, atol=1e-6)
    else:
        np.testing.assert_allclose(inner.fc1.weight.numpy(), ref.fc1.weight.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(inner.fc2.weight.numpy(), ref.fc2.weight.numpy(), rtol=1e-5, atol=1e-6)
    print(f"rank{dist.get_rank()} {mode} OK", flush=True)


if __name__ == '__main__':
    main(sys.argv[1])
