"""GPT-tiny under group-sharded stage 1/2/3 must match unsharded training (CPU gloo or world 1)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
from paddle.models.gpt import gpt_config, GPTForPretraining  # noqa: E402


def run(level, world, rank, reduce_dtype=None):
    cfg = gpt_config('gpt-tiny', hidden_dropout_prob=0.0)
    paddle.seed(1)
    ref = GPTForPretraining(cfg)
    paddle.seed(1)
    m = GPTForPretraining(cfg)
    ropt = paddle.optimizer.AdamW(1e-3, parameters=ref.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    opt = paddle.optimizer.AdamW(1e-3, parameters=m.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    m, opt, _ = dist.sharding.group_sharded_parallel(m, opt, level=level, segment_size=1024,
                                                      reduce_dtype=reduce_dtype)
    g = torch.Generator().manual_seed(0)
    for step in range(3):
        ids = torch.randint(0, cfg.vocab_size, (2 * world, 17), generator=g)
        x, y = paddle.to_tensor(ids[:, :-1]), paddle.to_tensor(ids[:, 1:])
        l = ref.loss(ref(x), y)
        l.backward()
        ropt.step()
        ropt.clear_grad()
        xs, ys = x[rank * 2:(rank + 1) * 2], y[rank * 2:(rank + 1) * 2]
        l2 = m._layers.loss(m(xs), ys)
        l2.backward()
        opt.step()
        opt.clear_grad()
    got = m.state_dict()
    for k, v in ref.state_dict().items():
        err = float((got[k]._t.float() - v._t.float()).abs().max())
        assert err < 5e-5, (level, k, err)
    print(f"rank{rank} gpt {level}{'' if reduce_dtype is None else '-' + reduce_dtype} OK", flush=True)


if __name__ == '__main__':
    level = sys.argv[1]
    rd = sys.argv[2] if len(sys.argv) > 2 else None
    if int(os.environ.get('WORLD_SIZE', '1')) > 1:
        dist.init_parallel_env()
    run(level, dist.get_world_size(), dist.get_rank(), rd)
