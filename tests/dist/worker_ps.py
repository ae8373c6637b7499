"""Parameter-server mode: 2 servers + 2 trainers (sync SGD) equal single-process full-batch SGD.
Launched with TRAINING_ROLE / PADDLE_* env per process (tests/test_distributed_cpu.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle  # noqa: E402
from paddle.distributed import fleet  # noqa: E402
from paddle.distributed.ps import DistributedEmbedding  # noqa: E402


class Net(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.emb = DistributedEmbedding(1000, 8, table_name='emb', init_range=0.5, seed=7)
        self.fc = paddle.nn.Linear(8, 1)

    def forward(self, ids):
        return self.fc(self.emb(ids).mean(1))


def main():
    fleet.init(fleet.PaddleCloudRoleMaker(is_collective=False))
    if fleet.is_server():
        fleet.init_server()
        fleet.run_server()
        print(f"server{fleet.server_index()} ps OK", flush=True)
        return
    fleet.init_worker()
    r, n = fleet.worker_index(), fleet.worker_num()
    rs = np.random.RandomState(0)
    ids_all = rs.randint(0, 1000, size=(8, 5)).astype('int64')
    ids_all[1, :2] = ids_all[0, :2]  # repeated rows inside and across trainers
    y_all = rs.randn(8, 1).astype('float32')
    paddle.seed(11)
    net = Net()
    s = fleet.DistributedStrategy()
    s.a_sync = False
    opt = fleet.distributed_optimizer(paddle.optimizer.SGD(learning_rate=0.2, parameters=net.parameters()), s)
    # reference: same initial rows (pulled) and dense init, trained on the full batch in-process
    uniq = np.unique(ids_all)
    net(paddle.to_tensor(ids_all[:1]))  # binds the table (creates it on the servers)
    init_rows = opt._client.pull_sparse('emb', torch.from_numpy(uniq))
    table = {int(i): init_rows[k].clone() for k, i in enumerate(uniq)}
    W = net.fc.weight._t.detach().clone()
    b = net.fc.bias._t.detach().clone()
    net.emb._pending = []
    lo, hi = r * 8 // n, (r + 1) * 8 // n
    for _ in range(4):
        loss = ((net(paddle.to_tensor(ids_all[lo:hi])) - paddle.to_tensor(y_all[lo:hi])) ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        # reference step on the full batch
        E = torch.stack([torch.stack([table[int(i)] for i in row]) for row in ids_all]).requires_grad_()
        Wr, br = W.clone().requires_grad_(), b.clone().requires_grad_()
        # each trainer's loss is the mean over its half; the server averages the two gradients
        lr_ = sum(((E[a:c].mean(1) @ Wr + br - torch.from_numpy(y_all[a:c])) ** 2).mean()
                  for a, c in ((0, 4), (4, 8))) / 2
        lr_.backward()
        with torch.no_grad():
            W -= 0.2 * Wr.grad
            b -= 0.2 * br.grad
            gE = E.grad
            acc = {}
            for rr in range(8):
                for cc in range(5):
                    i = int(ids_all[rr, cc])
                    acc[i] = acc.get(i, 0) + gE[rr, cc]
            for i, g in acc.items():
                table[i] = table[i] - 0.2 * g
    np.testing.assert_allclose(net.fc.weight._t.detach().numpy(), W.numpy(), atol=1e-5)
    np.testing.assert_allclose(net.fc.bias._t.detach().numpy(), b.numpy(), atol=1e-5)
    rows = opt._client.pull_sparse('emb', torch.from_numpy(uniq))
    ref = torch.stack([table[int(i)] for i in uniq])
    np.testing.assert_allclose(rows.numpy(), ref.numpy(), atol=1e-5)
    fleet.stop_worker()
    print(f"trainer{r} ps OK", flush=True)


if __name__ == '__main__':
    main()
