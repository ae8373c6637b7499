"""auto_parallel reshard transitions + distributed checkpoint resharding (gloo world 2)."""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
from paddle.distributed import ProcessMesh, Shard, Replicate, Partial  # noqa: E402


def main():
    dist.init_parallel_env()
    r = dist.get_rank()
    mesh = ProcessMesh([0, 1], dim_names=['x'])
    g = torch.arange(24, dtype=torch.float32).reshape(4, 6)
    full = paddle.to_tensor(g)
    s0 = dist.shard_tensor(full, mesh, [Shard(0)])
    assert s0.shape == [2, 6] and torch.equal(s0._t, g[2 * r:2 * r + 2])
    rep = dist.reshard(s0, mesh, [Replicate()])
    assert torch.equal(rep._t, g)
    s1 = dist.reshard(s0, mesh, [Shard(1)])
    assert torch.equal(s1._t, g[:, 3 * r:3 * r + 3]), s1._t
    p = dist.shard_tensor(full, mesh, [Partial()])
    pr = dist.reshard(p, mesh, [Replicate()])
    assert torch.equal(pr._t, g)
    ps = dist.reshard(p, mesh, [Shard(0)])
    assert torch.equal(ps._t, g[2 * r:2 * r + 2])
    un = dist.unshard_dtensor(s1)
    assert torch.equal(un._t, g)
    # checkpoint: save Shard(0), load into Shard(1) and into a replicated tensor
    d = os.environ['CKPT_DIR']
    dist.save_state_dict({'w': s0, 'step': 7}, d)
    tgt = dist.shard_tensor(paddle.zeros([4, 6]), mesh, [Shard(1)])
    sd = {'w': tgt, 'step': 0}
    dist.load_state_dict(sd, d)
    assert torch.equal(tgt._t, g[:, 3 * r:3 * r + 3]) and sd['step'] == 7
    plain = paddle.zeros([4, 6])
    dist.load_state_dict({'w': plain}, d)
    assert torch.equal(plain._t, g)
    print(f"rank{r} auto_parallel OK", flush=True)


if __name__ == '__main__':
    main()
