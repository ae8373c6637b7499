"""Watchdog: rank 1 skips a collective; rank 0's all_reduce must be reported (then both exit)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402


def main():
    dist.init_parallel_env()
    dist.watchdog.enable(timeout_s=1.0)
    r = dist.get_rank()
    x = paddle.ones([4])
    dist.all_reduce(x)
    assert float(x.sum()) == 8.0
    if r == 0:
        task = dist.all_reduce(x, sync_op=False)  # rank 1 never joins
        time.sleep(3.0)
        reps = dist.watchdog.reports()
        assert reps and 'all_reduce' in reps[0] and '(4,)' in reps[0], reps
        print("rank0 watchdog OK", flush=True)
        os._exit(0)
    else:
        time.sleep(4.0)
        print("rank1 watchdog OK", flush=True)
        os._exit(0)
    _ = task


if __name__ == '__main__':
    main()
