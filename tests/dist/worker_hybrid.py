"""TP (mp=2), SP and PP (pp=2) workers: results must equal the single-device computation."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.nn as nn  # noqa: E402
from paddle.distributed import fleet  # noqa: E402


def gather_full(t, axis):
    parts = []
    dist.all_gather(parts, t)
    return torch.cat([p._t for p in parts], axis)


def tp_test():
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': 1, 'mp_degree': 2, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    assert hcg.get_model_parallel_world_size() == 2
    V, H, F = 16, 8, 12
    paddle.seed(3 + hcg.get_model_parallel_rank())
    emb = fleet.meta_parallel.VocabParallelEmbedding(V, H)
    col = fleet.meta_parallel.ColumnParallelLinear(H, F, gather_output=False)
    row = fleet.meta_parallel.RowParallelLinear(F, H, input_is_parallel=True)
    ce = fleet.meta_parallel.ParallelCrossEntropy()
    col_gather = fleet.meta_parallel.ColumnParallelLinear(H, V, gather_output=False)
    ids = paddle.to_tensor(np.array([[1, 9, 15, 3]]))
    h = emb(ids)
    logits_sh = col_gather(row(paddle.nn.functional.relu(col(h))))
    loss = ce(logits_sh, ids.unsqueeze(-1)).mean()
    loss.backward()
    # single-device reference from gathered full weights
    We = gather_full(emb.weight, 0).detach().requires_grad_()
    W1 = gather_full(col.weight, 1).detach().requires_grad_()
    b1 = gather_full(col.bias, 0).detach().requires_grad_()
    W2 = gather_full(row.weight, 0).detach().requires_grad_()
    b2 = row.bias._t.detach().requires_grad_()
    W3 = gather_full(col_gather.weight, 1).detach().requires_grad_()
    b3 = gather_full(col_gather.bias, 0).detach().requires_grad_()
    x = We[ids._t]
    z = torch.relu(x @ W1 + b1) @ W2 + b2
    lg = z @ W3 + b3
    ref = torch.nn.functional.cross_entropy(lg.reshape(-1, V), ids._t.reshape(-1))
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-5, (float(loss), float(ref))
    r = hcg.get_model_parallel_rank()
    np.testing.assert_allclose(col.weight.grad.numpy(), W1.grad.chunk(2, 1)[r].numpy(), atol=1e-5)
    np.testing.assert_allclose(row.weight.grad.numpy(), W2.grad.chunk(2, 0)[r].numpy(), atol=1e-5)
    np.testing.assert_allclose(emb.weight.grad.numpy(), We.grad.chunk(2, 0)[r].numpy(), atol=1e-5)
    print(f"rank{dist.get_rank()} tp OK", flush=True)


def tpdp_test():
    """TP=2 x DP=2 (4 ranks): the dp replicas see different halves of the batch; the hybrid
    optimizer all-reduces their gradients over dp, so two SGD steps equal single-device training
    on the whole batch."""
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': 2, 'mp_degree': 2, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    r, dpr = hcg.get_model_parallel_rank(), hcg.get_data_parallel_rank()
    H, F = 8, 12
    paddle.seed(5)  # same full weights everywhere
    W1 = torch.randn(H, F) * 0.3
    W2 = torch.randn(F, H) * 0.3
    col = fleet.meta_parallel.ColumnParallelLinear(H, F, gather_output=False, has_bias=False)
    row = fleet.meta_parallel.RowParallelLinear(F, H, input_is_parallel=True, has_bias=False)
    with torch.no_grad():
        col.weight._t.copy_(W1.chunk(2, 1)[r])
        row.weight._t.copy_(W2.chunk(2, 0)[r])
    net = nn.LayerList([col, row])
    model = fleet.distributed_model(net)
    opt = fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.5, parameters=net.parameters()))
    g = torch.Generator().manual_seed(9)
    ref1, ref2 = W1.clone().requires_grad_(), W2.clone().requires_grad_()
    for step in range(2):
        X = torch.randn(8, H, generator=g)
        T = torch.randn(8, H, generator=g)
        xs, ts = X[4 * dpr:4 * dpr + 4], T[4 * dpr:4 * dpr + 4]
        y = row(paddle.nn.functional.relu(col(paddle.to_tensor(xs))))
        loss = ((y - paddle.to_tensor(ts)) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        lref = ((torch.relu(X @ ref1) @ ref2 - T) ** 2).mean()
        lref.backward()
        with torch.no_grad():
            ref1 -= 0.5 * ref1.grad
            ref2 -= 0.5 * ref2.grad
            ref1.grad = None
            ref2.grad = None
    np.testing.assert_allclose(col.weight.numpy(), ref1.detach().chunk(2, 1)[r].numpy(), atol=1e-5)
    np.testing.assert_allclose(row.weight.numpy(), ref2.detach().chunk(2, 0)[r].numpy(), atol=1e-5)
    print(f"rank{dist.get_rank()} tpdp OK", flush=True)


def sp_test():
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': 1, 'mp_degree': 2, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=s)
    from paddle.distributed.fleet.utils.sequence_parallel_utils import (ScatterOp, GatherOp,
                                                                        ColumnSequenceParallelLinear,
                                                                        RowSequenceParallelLinear)
    paddle.seed(11)
    S, B, H = 8, 2, 4
    x_full = paddle.randn([S, B, H])
    x_full.stop_gradient = False
    paddle.seed(20 + dist.get_rank())
    col = ColumnSequenceParallelLinear(H, 6, has_bias=True)
    row = RowSequenceParallelLinear(6, H, has_bias=True)
    xs = ScatterOp.apply(x_full)
    y = GatherOp.apply(row(col(xs)))
    y.sum().backward()
    W1 = gather_full(col.weight, 1)
    b1 = gather_full(col.bias, 0)
    W2 = gather_full(row.weight, 0)
    ref = (x_full._t @ W1 + b1) @ W2 + row.bias._t
    np.testing.assert_allclose(y.numpy(), ref.detach().numpy(), atol=1e-5)
    print(f"rank{dist.get_rank()} sp OK", flush=True)


class Block(nn.Layer):
    def __init__(self, d):
        super().__init__()
        self.fc = nn.Linear(d, d)

    def forward(self, x):
        return paddle.tanh(self.fc(x))


def pp_test(virtual=1, acc=4, tag=None, sched='1F1B'):
    world = int(os.environ['WORLD_SIZE'])
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': 1, 'mp_degree': 1, 'pp_degree': world}
    s.pipeline_configs = {'accumulate_steps': acc, 'micro_batch_size': 8 // acc, 'schedule_mode': sched}
    fleet.init(is_collective=True, strategy=s)
    d = 6
    nblk = 2 * world * virtual
    descs = [fleet.meta_parallel.LayerDesc(Block, d) for _ in range(nblk)]
    loss_fn = lambda out, y: ((out - y) ** 2).mean()  # noqa: E731
    # build the full reference on every rank with the same seed sequence
    paddle.seed(5)
    full = [Block(d) for _ in range(nblk)]
    paddle.seed(5)
    pl = fleet.meta_parallel.PipelineLayer(descs, num_stages=world, loss_fn=loss_fn,
                                           num_virtual_pipeline_stages=virtual)
    stage = fleet.get_hybrid_communicate_group().get_stage_id()
    # copy the reference weights of this stage's blocks so both start equal
    owned = [i for lo, hi in pl._chunk_ranges for i in range(lo, hi)]
    for blk, gi in zip(pl.run_function, owned):
        src = full[gi]
        blk.fc.weight.set_value(src.fc.weight)
        blk.fc.bias.set_value(src.fc.bias)
    model = fleet.distributed_model(pl)
    opt = paddle.optimizer.SGD(learning_rate=0.1, parameters=pl.parameters())
    x = paddle.to_tensor(np.random.RandomState(0).randn(8, d).astype('float32'))
    y = paddle.to_tensor(np.random.RandomState(1).randn(8, d).astype('float32'))
    if sched == 'ZBH1':
        from paddle.distributed.fleet.meta_parallel import zero_bubble_utils as zb
        calls = []
        orig = zb.SplitBwLinear.backward
        zb.SplitBwLinear.backward = staticmethod(lambda ctx, dy: (calls.append(1), orig(ctx, dy))[1])
    loss = model.train_batch([x, y], opt)
    if sched == 'ZBH1':
        zb.SplitBwLinear.backward = orig
        assert calls and zb.WeightGradStore.pending() == 0  # backward really ran split (B, then W)
    # reference: same micro-batches, mean of per-micro-batch losses
    ropt = paddle.optimizer.SGD(learning_rate=0.1, parameters=[p for b in full for p in b.parameters()])
    tot = 0.0
    mbs = 8 // acc
    for mb in range(acc):
        h = x[mb * mbs:(mb + 1) * mbs]
        for b in full:
            h = b(h)
        l = loss_fn(h, y[mb * mbs:(mb + 1) * mbs]) / acc
        l.backward()
        tot += float(l)
    ropt.step()
    assert abs(float(loss) - tot) < 1e-5, (float(loss), tot)
    for blk, gi in zip(pl.run_function, owned):
        np.testing.assert_allclose(blk.fc.weight.numpy(), full[gi].fc.weight.numpy(), atol=1e-5)
    tag = tag or ('pp' if virtual == 1 else 'vpp')
    if virtual > 1 and sched == '1F1B':
        # the reference's choice (fleet/model.py:168): FthenB for pp <= acc < 2 pp, else 1F1B
        want = 'interleaved_fthenb' if acc < 2 * world else 'interleaved_1f1b'
        assert model.schedule == want, (model.schedule, want)
    print(f"rank{dist.get_rank()} {tag} OK stage{stage}", flush=True)


if __name__ == '__main__':
    {'tp': tp_test, 'sp': sp_test, 'pp': pp_test, 'vpp': lambda: pp_test(2), 'vpp8': lambda: pp_test(2, 8, 'vpp8'),
     'tpdp': tpdp_test, 'zbh1': lambda: pp_test(1, 4, 'zbh1', 'ZBH1'),
     'zbh1_8': lambda: pp_test(1, 8, 'zbh1_8', 'ZBH1')}[sys.argv[1]]()
