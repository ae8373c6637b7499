"""Llama-2 (tiny) hybrid parallel TP=2 x PP=2 (4 gloo ranks): pipeline train_batch loss and the
updated weight shards equal a single-device LlamaForCausalLM trained on the same batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
from paddle.distributed import fleet  # noqa: E402
from paddle.models.llama import llama_config, LlamaForCausalLM  # noqa: E402
from paddle.models import llama_hybrid as LH  # noqa: E402


def main():
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': 1, 'mp_degree': 2, 'pp_degree': 2}
    s.pipeline_configs = {'accumulate_steps': 2, 'micro_batch_size': 2}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    mp_rank, stage = hcg.get_model_parallel_rank(), hcg.get_stage_id()
    cfg = llama_config('llama-tiny', num_hidden_layers=4, tie_word_embeddings=False, vocab_size=256)
    paddle.seed(7)
    full = LlamaForCausalLM(cfg)  # same dense init on every rank
    pipe = LH.LlamaForCausalLMPipe(cfg, num_stages=2, topology=hcg.topology())
    LH.load_full_weights(pipe, full, mp_rank, 2)
    model = fleet.distributed_model(pipe)
    opt = paddle.optimizer.SGD(learning_rate=0.5, parameters=pipe.parameters())
    rs = np.random.RandomState(0)
    ids = rs.randint(0, cfg.vocab_size, size=(4, 17)).astype('int64')
    x, y = paddle.to_tensor(ids[:, :-1]), paddle.to_tensor(ids[:, 1:])
    loss = model.train_batch([x, y], opt)
    # reference: two micro-batches of 2, mean of their token-mean losses
    ropt = paddle.optimizer.SGD(learning_rate=0.5, parameters=full.parameters())
    tot = 0.0
    for mb in range(2):
        sl = slice(2 * mb, 2 * mb + 2)
        lr_ = full.loss(full(x[sl]), y[sl]) / 2
        lr_.backward()
        tot += float(lr_)
    ropt.step()
    assert abs(float(loss) - tot) < 2e-4, (float(loss), tot)
    # the updated shards equal the shards of the updated dense weights
    check = LH.LlamaForCausalLMPipe(cfg, num_stages=2, topology=hcg.topology())
    LH.load_full_weights(check, full, mp_rank, 2)
    for (n, a), (_, b) in zip(pipe.named_parameters(), check.named_parameters()):
        np.testing.assert_allclose(a.numpy(), b.numpy(), atol=2e-4, err_msg=n)
    print(f"rank{dist.get_rank()} llama hybrid OK stage{stage} mp{mp_rank}", flush=True)


if __name__ == '__main__':
    main()
