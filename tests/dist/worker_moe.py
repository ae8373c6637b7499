"""Expert-parallel MoE (world 2, 2 local experts each) equals a single-process MoE holding all 4
experts with the same gate, forward and input gradients.  argv[1] == 'ffn': Linear-GELU-Linear
experts, which run as batched GEMMs with the one-index receive-buffer regroup."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
from paddle.incubate.distributed.models.moe import MoELayer, NaiveGate  # noqa: E402


class Expert(paddle.nn.Layer):
    def __init__(self, d):
        super().__init__()
        self.fc = paddle.nn.Linear(d, d)

    def forward(self, x):
        return paddle.nn.functional.relu(self.fc(x))


class FFN(paddle.nn.Layer):
    def __init__(self, d):
        super().__init__()
        self.fc1 = paddle.nn.Linear(d, 2 * d)
        self.fc2 = paddle.nn.Linear(2 * d, d)

    def forward(self, x):
        return self.fc2(paddle.nn.functional.gelu(self.fc1(x)))


def main():
    ffn = len(sys.argv) > 1 and sys.argv[1] == 'ffn'
    dist.init_parallel_env()
    r, W, d = dist.get_rank(), 2, 8
    paddle.seed(0)
    all_exp = [(FFN if ffn else Expert)(d) for _ in range(4)]
    gate = NaiveGate(d, 4, 1, topk=2)
    ref = MoELayer(d, all_exp, gate=gate)
    group = dist.new_group([0, 1])
    local = MoELayer(d, [all_exp[2 * r], all_exp[2 * r + 1]], gate={'type': 'naive', 'top_k': 2}, moe_group=group)
    local.gate.gate.weight.set_value(gate.gate.weight)
    local.gate.gate.bias.set_value(gate.gate.bias)
    g = torch.Generator().manual_seed(r)
    x = paddle.to_tensor(torch.randn(2, 5, d, generator=g))
    x.stop_gradient = False
    y = local(x)
    x2 = paddle.to_tensor(x.numpy())
    x2.stop_gradient = False
    y2 = ref(x2)
    assert float((y - y2).abs().max()) < 1e-5, float((y - y2).abs().max())
    if ffn:
        assert local._grouped.get(True), local._grouped  # the batched-GEMM path ran
    y.sum().backward()
    y2.sum().backward()
    assert float((x.grad - x2.grad).abs().max()) < 1e-5
    print(f"rank{r} moe OK", flush=True)


if __name__ == '__main__':
    main()
