"""Pipeline-shared weights under the fleet sharding axis (PP=2 x sharding=2, 4 gloo ranks): a
SharedLayerDesc embedding used as the input embedding on stage 0 and as the tied output head on
stage 1.  Two AdamW steps of train_batch must equal one device training the tied model on the
whole batch, with both stages' copies of the shared weight identical.
(reference: pp_layers.py SharedLayerDesc:76 / allreduce_shared_weight_gradients,
dygraph_sharding_optimizer.py:44.)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.nn as nn  # noqa: E402
import paddle.nn.functional as F  # noqa: E402
from paddle.distributed import fleet  # noqa: E402
from paddle.distributed.fleet.meta_parallel import LayerDesc, PipelineLayer, SharedLayerDesc  # noqa: E402

V, E = 32, 16


def head(layer, x):
    return paddle.matmul(x, layer.weight, transpose_y=True)


def loss_fn(logits, label):
    return F.cross_entropy(logits.reshape([-1, V]), label.reshape([-1]))


def adamw(params, clip):
    return paddle.optimizer.AdamW(learning_rate=0.01, parameters=params, weight_decay=0.1, epsilon=1e-3,
                                  grad_clip=paddle.nn.ClipGradByGlobalNorm(clip) if clip else None)


def main():
    clip = float(os.environ.get('CLIP', '0'))
    s = fleet.DistributedStrategy()
    shard = os.environ.get('SHARD', '1') == '1'  # else the same 2-way split as a plain dp axis
    s.hybrid_configs = {'dp_degree': 1 if shard else 2, 'mp_degree': 1, 'pp_degree': 2,
                        'sharding_degree': 2 if shard else 1}
    s.pipeline_configs = {'accumulate_steps': 2, 'micro_batch_size': 2}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    stage = hcg.get_stage_id()
    sh_rank = hcg.get_sharding_parallel_rank() if shard else hcg.get_data_parallel_rank()
    paddle.seed(7)
    emb, l1, l2 = nn.Embedding(V, E), nn.Linear(E, E), nn.Linear(E, E)  # the single-device model
    descs = [SharedLayerDesc('embed', nn.Embedding, None, 'weight', V, E), LayerDesc(nn.Linear, E, E),
             LayerDesc(nn.Tanh), LayerDesc(nn.Linear, E, E), LayerDesc(nn.Tanh),
             SharedLayerDesc('embed', nn.Embedding, head, 'weight', V, E)]
    pipe = PipelineLayer(layers=descs, num_stages=2, topology=hcg.topology(), loss_fn=loss_fn)
    lin = [f for f in pipe.run_function if isinstance(f, nn.Linear)]
    assert len(lin) == 1
    pipe.shared_layers['embed'].weight.set_value(emb.weight)
    src = l1 if stage == 0 else l2
    lin[0].weight.set_value(src.weight)
    lin[0].bias.set_value(src.bias)
    model = fleet.distributed_model(pipe)
    opt = fleet.distributed_optimizer(adamw(pipe.parameters(), clip))
    if shard:  # the shared weight has a unit of its own
        shared_units = list(opt._shared_units())
        assert len(shared_units) == 1 and shared_units[0][1].params[0] is pipe.shared_layers['embed'].weight
    rs = np.random.RandomState(0)
    ropt = adamw(list(emb.parameters()) + list(l1.parameters()) + list(l2.parameters()), clip)
    for step in range(2):
        ids = rs.randint(0, V, size=(8, 6)).astype('int64')
        lab = rs.randint(0, V, size=(8, 6)).astype('int64')
        mine = slice(4 * sh_rank, 4 * sh_rank + 4)  # the sharding axis splits the global batch
        loss = model.train_batch([paddle.to_tensor(ids[mine]), paddle.to_tensor(lab[mine])], opt)
        assert np.isfinite(float(loss))
        for mb in range(4):  # single device: 4 micro-batches of 2, mean over all of them
            sl = slice(2 * mb, 2 * mb + 2)
            x = emb(paddle.to_tensor(ids[sl]))
            x = paddle.tanh(l2(paddle.tanh(l1(x))))
            (loss_fn(head(emb, x), paddle.to_tensor(lab[sl])) / 4).backward()
        ropt.step()
        ropt.clear_grad()
    np.testing.assert_allclose(pipe.shared_layers['embed'].weight.numpy(), emb.weight.numpy(), atol=2e-5, rtol=1e-4)
    np.testing.assert_allclose(lin[0].weight.numpy(), src.weight.numpy(), atol=2e-5, rtol=1e-4)
    np.testing.assert_allclose(lin[0].bias.numpy(), src.bias.numpy(), atol=2e-5, rtol=1e-4)
    print(f"rank{dist.get_rank()} pp2 {'sharding2' if shard else 'dp2'} shared-weight OK stage{stage} sh{sh_rank}", flush=True)


if __name__ == '__main__':
    main()
