"""fleet.distributed_scaler (2 gloo ranks): an overflow on ONE rank makes every rank skip the
step and halve the loss scale (reference: fleet/scaler.py distributed_scaler)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
from paddle.distributed import fleet  # noqa: E402


def main():
    s = fleet.DistributedStrategy()
    s.hybrid_configs = {'dp_degree': 2, 'mp_degree': 1, 'pp_degree': 1}
    fleet.init(is_collective=True, strategy=s)
    rank = dist.get_rank()
    paddle.seed(1)
    lin = paddle.nn.Linear(4, 2)
    w0 = lin.weight.numpy().copy()
    opt = fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.1, parameters=lin.parameters()))
    scaler = fleet.distributed_scaler(paddle.amp.GradScaler(init_loss_scaling=1024.0))
    x = paddle.ones([3, 4]) * (float('inf') if rank == 1 else 1.0)
    loss = lin(x).sum()
    scaler.scale(loss).backward()
    scaler.step(opt)
    scaler.update()
    np.testing.assert_array_equal(lin.weight.numpy(), w0)  # skipped on BOTH ranks
    assert scaler.get_init_loss_scaling() == 512.0, scaler.get_init_loss_scaling()
    print(f"rank{rank} scaler OK", flush=True)


if __name__ == '__main__':
    main()
