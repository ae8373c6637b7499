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


def _train(level, alias, reduce_dtype=None, steps=3, momentum=False, segment_size=1024):
    cfg = gpt_config('gpt-tiny', hidden_dropout_prob=0.0)
    paddle.seed(3)
    m = GPTForPretraining(cfg)
    if momentum:
        opt = paddle.optimizer.Momentum(1e-2, momentum=0.9, parameters=m.parameters(), use_nesterov=True,
                                        weight_decay=1e-4)
    else:
        opt = paddle.optimizer.AdamW(1e-3, parameters=m.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    m, opt, _ = dist.sharding.group_sharded_parallel(m, opt, level=level, segment_size=segment_size, alias=alias,
                                                      reduce_dtype=reduce_dtype)
    g = torch.Generator().manual_seed(0)
    losses = []
    for _ in range(steps):
        b = torch.randint(0, cfg.vocab_size, (2, 17), generator=g)
        x, y = paddle.to_tensor(b[:, :-1]), paddle.to_tensor(b[:, 1:])
        loss = m._layers.loss(m(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    eng = m.__dict__['_engine']
    eng._test_wemb = m._layers.gpt.embeddings.word_embeddings.weight
    return losses, m.state_dict(), eng


import pytest  # noqa: E402


@pytest.mark.parametrize("level", ['os', 'os_g', 'p_g_os'])
@pytest.mark.parametrize("momentum", [False, True])
@pytest.mark.parametrize("segment_size", [1024, 4096])
def test_world1_alias_off_matches_alias_on(level, momentum, segment_size):
    """alias=False runs the multi-rank path (release / gather / re-materialise / shard copies,
    async stage-1/2 parameter gathers) on one rank: bit-identical to the aliased fast path."""
    l1, s1, e1 = _train(level, True, momentum=momentum, segment_size=segment_size)
    l0, s0, e0 = _train(level, False, momentum=momentum, segment_size=segment_size)
    # the tied word embedding always sits in a persistent unit (used by the LM head outside its layer)
    emb = [u for u in e0.units if any(p is e0._test_wemb for p in u.params)]
    assert len(emb) == 1 and emb[0].persistent
    assert e1.alias and not e0.alias
    if level == 'p_g_os':
        assert any(not u.persistent for u in e0.units)  # something is really released
    assert l1 == l0
    for k in s1:
        np.testing.assert_array_equal(s0[k].numpy(), s1[k].numpy(), err_msg=k)


def test_world1_fp32_reduce_dtype_arena():
    import paddle.nn as nn
    l1, s1, e1 = _train('p_g_os', False)
    l0, s0, e0 = _train('p_g_os', False, reduce_dtype='float32')
    assert all(a['grad'].dtype == torch.float32 for a in e0.arenas.values())
    np.testing.assert_allclose(l0, l1, rtol=1e-6)
    with pytest.raises(ValueError):
        _train('os', False, reduce_dtype='int8', steps=1)
