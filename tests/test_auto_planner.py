"""Rule-based auto-parallel planner (reference: python/paddle/distributed/auto_parallel/static/
tuner/rule_based_tuner.py): pattern matching on the recorded op graph (single process)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle  # noqa: E402
from paddle.distributed.auto_parallel.static.planner import RuleBasedPlanner  # noqa: E402


class _Mesh:
    def __init__(self, shape, names):
        self.shape, self.dim_names, self.ndim = list(shape), list(names), len(shape)


def _kinds(p):
    return [k for k, _ in p.patterns]


def test_mlp_stack_alternates_column_row():
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.GELU(), paddle.nn.Linear(16, 8), paddle.nn.Tanh(),
                               paddle.nn.Linear(8, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 4))
    p = RuleBasedPlanner(_Mesh([2], ['mp'])).plan(net, paddle.randn([3, 8]))
    assert _kinds(p) == ['ffn', 'ffn']
    assert str(p['0.weight'][0]) == 'Shard(dim=1)' and str(p['2.weight'][0]) == 'Shard(dim=0)'
    assert str(p['4.weight'][0]) == 'Shard(dim=1)' and str(p['6.weight'][0]) == 'Shard(dim=0)'
    assert '2.bias' not in p  # the row-parallel bias stays replicated


def test_transformer_layer_attention_and_ffn_on_2d_mesh():
    enc = paddle.nn.TransformerEncoderLayer(16, 4, 32, dropout=0.0)
    p = RuleBasedPlanner(_Mesh([2, 2], ['dp', 'mp'])).plan(enc, paddle.randn([2, 5, 16]))
    assert sorted(_kinds(p)) == ['attention', 'ffn']
    q = p['self_attn.q_proj.weight']
    assert str(q[0]) == 'Replicate()' and str(q[1]) == 'Shard(dim=1)'
    assert str(p['self_attn.out_proj.weight'][1]) == 'Shard(dim=0)'
    assert 'norm1.weight' not in p


def test_indivisible_and_fused_blocks_stay_replicated():
    net = paddle.nn.Sequential(paddle.nn.Linear(6, 7), paddle.nn.ReLU(), paddle.nn.Linear(7, 6))
    assert len(RuleBasedPlanner(_Mesh([2], ['mp'])).plan(net, paddle.randn([3, 6]))) == 0

    class Fused(paddle.nn.Layer):  # a fused qkv split by chunk (no SPMD rule): not planned
        def __init__(self):
            super().__init__()
            self.qkv = paddle.nn.Linear(8, 24)
            self.o = paddle.nn.Linear(8, 8)

        def forward(self, x):
            q, k, v = paddle.chunk(self.qkv(x), 3, axis=-1)
            return self.o(paddle.nn.functional.softmax(q @ k.transpose([0, 2, 1]), -1) @ v)
    assert len(RuleBasedPlanner(_Mesh([2], ['mp'])).plan(Fused(), paddle.randn([2, 3, 8]))) == 0
