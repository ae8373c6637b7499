"""paddle.distributed.rpc between two workers (launched by torch.distributed.run)."""
import operator
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

import paddle.distributed.rpc as rpc  # noqa: E402


def scaled_sum(t, k=1.0):
    return (t * k).sum()


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    port = int(sys.argv[1])
    os.environ['PADDLE_WORKER_ENDPOINT'] = f"127.0.0.1:{port + 1 + rank}"
    rpc.init_rpc(f"worker{rank}", rank=rank, world_size=world, master_endpoint=f"127.0.0.1:{port}")
    infos = rpc.get_all_worker_infos()
    assert [i.name for i in infos] == [f"worker{r}" for r in range(world)], infos
    assert rpc.get_current_worker_info().rank == rank
    peer = f"worker{(rank + 1) % world}"
    assert rpc.get_worker_info(peer).rank == (rank + 1) % world
    assert rpc.rpc_sync(peer, operator.add, args=(2, 3 + rank)) == 5 + rank
    fut = rpc.rpc_async(peer, scaled_sum, args=(torch.arange(4.0),), kwargs={'k': 2.0})
    assert float(fut.wait()) == 12.0
    rpc.shutdown()
    print("rpc OK", flush=True)


if __name__ == '__main__':
    main()
