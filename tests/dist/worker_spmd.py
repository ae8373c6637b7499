"""SPMD propagation (semi-auto parallel) on gloo world 2: column/row-parallel MLP, data parallel
and shape ops give the single-process values and gradients."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.nn.functional as F  # noqa: E402
from paddle.distributed import ProcessMesh, Shard, Replicate, Partial  # noqa: E402


def close(a, b, tol=1e-5, what=''):
    a = a._t.detach() if hasattr(a, '_t') else a
    b = b._t.detach() if hasattr(b, '_t') else b
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = (a - b).abs().max().item()
    assert err < tol, (what, err)


def main():
    dist.init_parallel_env()
    r = dist.get_rank()
    mesh = ProcessMesh([0, 1], dim_names=['x'])
    rs = np.random.RandomState(0)
    x_np = rs.randn(4, 8).astype('float32')
    w1_np = rs.randn(8, 6).astype('float32')
    w2_np = rs.randn(6, 8).astype('float32')

    # --- tensor parallel: W1 column-parallel (Shard(1)), W2 row-parallel (Shard(0))
    x = paddle.to_tensor(x_np, stop_gradient=False)
    w1 = dist.shard_tensor(paddle.create_parameter([8, 6], 'float32'), mesh, [Shard(1)])
    w2 = dist.shard_tensor(paddle.create_parameter([6, 8], 'float32'), mesh, [Shard(0)])
    with torch.no_grad():
        w1._t.copy_(torch.from_numpy(w1_np[:, 3 * r:3 * r + 3]))
        w2._t.copy_(torch.from_numpy(w2_np[3 * r:3 * r + 3]))
    h = F.relu(paddle.matmul(x, w1))
    assert h.placements[0] == Shard(1), h.placements
    y = paddle.matmul(h, w2)
    assert y.placements[0] == Partial(), y.placements
    loss = (y * y).sum()  # the non-linear consumer resolves the partial sum (all-reduce)
    loss.backward()
    # reference
    xr = torch.from_numpy(x_np).requires_grad_()
    w1r = torch.from_numpy(w1_np).requires_grad_()
    w2r = torch.from_numpy(w2_np).requires_grad_()
    lr = ((torch.relu(xr @ w1r) @ w2r) ** 2).sum()
    lr.backward()
    close(loss, lr.detach(), 1e-3, 'tp loss')
    close(w1._t.grad, w1r.grad[:, 3 * r:3 * r + 3], 1e-3, 'tp dW1 (column shard)')
    close(w2._t.grad, w2r.grad[3 * r:3 * r + 3], 1e-3, 'tp dW2 (row shard)')
    close(x._t.grad, xr.grad, 1e-3, 'tp dx (replicated input, all-reduced)')

    # --- data parallel: batch-sharded input, replicated weight; mean over the global batch
    w = dist.shard_tensor(paddle.create_parameter([8, 6], 'float32'), mesh, [Replicate()])
    with torch.no_grad():
        w._t.copy_(torch.from_numpy(w1_np))
    xb = dist.shard_tensor(paddle.to_tensor(x_np), mesh, [Shard(0)])
    out = paddle.matmul(xb, w)
    assert out.placements[0] == Shard(0)
    l2 = (out * out).mean()
    assert l2.placements[0] == Partial(), l2.placements
    l2.backward()
    wr = torch.from_numpy(w1_np).requires_grad_()
    lr2 = ((torch.from_numpy(x_np) @ wr) ** 2).mean()
    lr2.backward()
    close(dist.reshard(l2, mesh, [Replicate()]), lr2.detach(), 1e-4, 'dp loss')
    close(w._t.grad, wr.grad, 1e-4, 'dp dW (all-reduced)')

    # --- shape / norm ops keep or re-derive placements
    t = dist.shard_tensor(paddle.to_tensor(np.arange(48, dtype='float32').reshape(2, 4, 6)), mesh, [Shard(0)])
    tt = paddle.transpose(t, [1, 0, 2])
    assert tt.placements[0] == Shard(1), tt.placements
    rr = paddle.reshape(t, [8, 6])
    assert rr.placements[0] == Shard(0) and list(rr._t.shape) == [4, 6], (rr.placements, rr._t.shape)
    sm = F.softmax(dist.shard_tensor(paddle.to_tensor(x_np), mesh, [Shard(1)]), axis=-1)
    assert sm.placements[0] == Replicate()
    close(sm, torch.softmax(torch.from_numpy(x_np), -1), 1e-5, 'softmax over a sharded axis')
    s0 = paddle.sum(dist.shard_tensor(paddle.to_tensor(x_np), mesh, [Shard(1)]), axis=1)
    assert s0.placements[0] == Partial()
    close(dist.reshard(s0, mesh, [Replicate()]), torch.from_numpy(x_np).sum(1), 1e-4, 'sum over sharded axis')
    print(f"rank{r} spmd OK", flush=True)


if __name__ == '__main__':
    main()
