"""Single-rank group-sharded training (arena-aliased units) incl. gradient accumulation."""
import numpy as np
import torch

import paddle
import paddle.distributed as dist
from paddle.models.gpt import gpt_config, GPTForPretraining


def test_world1_sharding_grad_accumulation_matches_plain():
    cfg = gpt_config('gpt-tiny', hidden_dropout_prob=0.0)
    paddle.seed(3)
    ref = GPTForPretraining(cfg)
    paddle.seed(3)
    m = GPTForPretraining(cfg)
    ropt = paddle.optimizer.AdamW(1e-3, parameters=ref.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    opt = paddle.optimizer.AdamW(1e-3, parameters=m.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    m, opt, _ = dist.sharding.group_sharded_parallel(m, opt, level='p_g_os', segment_size=1024)
    g = torch.Generator().manual_seed(0)
    for _ in range(2):
        ids = [torch.randint(0, cfg.vocab_size, (2, 17), generator=g) for _ in range(2)]
        for b in ids:  # two micro-batches accumulate before one step
            x, y = paddle.to_tensor(b[:, :-1]), paddle.to_tensor(b[:, 1:])
            ref.loss(ref(x), y).backward()
            m._layers.loss(m(x), y).backward()
        ropt.step()
        ropt.clear_grad()
        opt.step()
        opt.clear_grad()
    got = m.state_dict()
    for k, v in ref.state_dict().items():
        np.testing.assert_allclose(got[k].numpy(), v.numpy(), atol=5e-5, err_msg=k)
