"""Llama-2 (tiny) hybrid parallel TP=2 x PP=2 x sharding=2 (8 gloo ranks): two AdamW steps of
pipeline train_batch with the sharding axis as a data-parallel axis (each sharding rank trains on
its half of the global batch) must equal a single-device LlamaForCausalLM trained on the whole
batch, and each sharding rank must hold half of the fp32 master weights / moments.
(reference: dygraph_sharding_optimizer.py:44 — the fleet sharding axis.)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
from paddle.distributed import fleet  # noqa: E402
from paddle.models.llama import llama_config, LlamaForCausalLM  # noqa: E402
from paddle.models import llama_hybrid as LH  # noqa: E402


def adamw(params, clip):
    return paddle.optimizer.AdamW(learning_rate=0.01, parameters=params, weight_decay=0.1, epsilon=1e-3,
                                  grad_clip=paddle.nn.ClipGradByGlobalNorm(clip) if clip else None)


def main():
    clip = float(os.environ.get('CLIP', '0'))
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': 1, 'mp_degree': 2, 'pp_degree': 2, 'sharding_degree': 2}
    s.pipeline_configs = {'accumulate_steps': 2, 'micro_batch_size': 2}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    mp_rank, stage, sh_rank = hcg.get_model_parallel_rank(), hcg.get_stage_id(), hcg.get_sharding_parallel_rank()
    cfg = llama_config('llama-tiny', num_hidden_layers=4, tie_word_embeddings=False, vocab_size=256)
    paddle.seed(7)
    full = LlamaForCausalLM(cfg)  # same dense init on every rank
    pipe = LH.LlamaForCausalLMPipe(cfg, num_stages=2, topology=hcg.topology())
    LH.load_full_weights(pipe, full, mp_rank, 2)
    model = fleet.distributed_model(pipe)
    opt = fleet.distributed_optimizer(adamw(pipe.parameters(), clip))
    from paddle.distributed.fleet.meta_optimizers import DygraphShardingOptimizer
    assert isinstance(opt, DygraphShardingOptimizer)
    # sharded optimizer state: this rank's arenas hold ~half of the local parameters
    local = sum(p._t.numel() for p in pipe.parameters())
    held = sum(a['master'].numel() for a in opt.engine.arenas.values())
    assert held <= local // 2 + 64 * 2 * len(opt.engine.units), (held, local)
    assert held >= local // 2, (held, local)
    rs = np.random.RandomState(0)
    ropt = adamw(full.parameters(), clip)
    for step in range(2):
        ids = rs.randint(0, cfg.vocab_size, size=(8, 17)).astype('int64')
        mine = ids[4 * sh_rank:4 * sh_rank + 4]  # the sharding axis splits the global batch
        x, y = paddle.to_tensor(mine[:, :-1]), paddle.to_tensor(mine[:, 1:])
        loss = model.train_batch([x, y], opt)
        # reference: 4 micro-batches of 2 (2 per sharding rank), mean over all of them
        X, Y = paddle.to_tensor(ids[:, :-1]), paddle.to_tensor(ids[:, 1:])
        tot = 0.0
        for mb in range(4):
            sl = slice(2 * mb, 2 * mb + 2)
            lr_ = full.loss(full(X[sl]), Y[sl]) / 4
            lr_.backward()
            tot += float(lr_)
        ropt.step()
        ropt.clear_grad()
        # this sharding rank's loss covers its own half of the batch only
        assert np.isfinite(float(loss))
    check = LH.LlamaForCausalLMPipe(cfg, num_stages=2, topology=hcg.topology())
    LH.load_full_weights(check, full, mp_rank, 2)
    for (n, a), (_, b) in zip(pipe.named_parameters(), check.named_parameters()):
        np.testing.assert_allclose(a.numpy(), b.numpy(), atol=3e-4, rtol=1e-3, err_msg=n)
    print(f"rank{dist.get_rank()} llama tp2 pp2 sharding2 OK stage{stage} mp{mp_rank} sh{sh_rank}", flush=True)


if __name__ == '__main__':
    main()
