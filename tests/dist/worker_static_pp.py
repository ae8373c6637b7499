"""Static Program pipeline parallelism over gloo ranks (reference: fleet static pipeline optimizer;
ops placed with static.device_guard('gpu:N'), pipeline_configs accumulate_steps micro-batches).
argv[1]: schedule ('1F1B' / 'FThenB' / 'ZBH1': zero bubble, weight gradients deferred behind the
input-gradient sends / 'VPP': 2 virtual stages per rank, a chain of 2 * pp device_guard stages run in
the interleaved 1F1B order); argv[2]: 'pp' (pp = world), 'ppdp' (pp 2 x dp 2), 'ppamp'
(pp = world + static AMP fp16 with dynamic loss scaling whose first step overflows: every stage must
skip it together) or 'ppgm' (pp = world + gradient merge k_steps 2: one update per two runs).
Every rank builds the same program (same seed); after 3 steps each stage's parameters must equal a
single-process run on the full batch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import paddle  # noqa: E402
import paddle.distributed as dist  # noqa: E402
import paddle.static as static  # noqa: E402
from paddle.distributed import fleet  # noqa: E402


def build(stages, opt_fn):
    paddle.seed(11)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 6], 'float32')
        y = static.data('y', [None, 1], 'int64')
        with static.device_guard('gpu:0'):
            h = static.nn.fc(x, 12, activation='relu')
            skip = static.nn.fc(x, 5)  # crosses two boundaries when there are 3 stages
        with static.device_guard(f'gpu:{min(1, stages - 1)}'):
            h = static.nn.fc(h, 10, activation='tanh')
        with static.device_guard(f'gpu:{stages - 1}'):
            z = paddle.concat([h, skip], axis=1)
            logits = static.nn.fc(z, 3)
            loss = paddle.nn.functional.cross_entropy(logits, y)
        opt_fn().minimize(loss)
    return main, startup, loss


def build_chain(C, opt_fn):
    """C device_guard stages, one fc each (the last one the head): the VPP layout."""
    paddle.seed(11)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 6], 'float32')
        y = static.data('y', [None, 1], 'int64')
        h = x
        for c in range(C):
            with static.device_guard(f'gpu:{c}'):
                if c < C - 1:
                    h = static.nn.fc(h, 8, activation='tanh')
                else:
                    logits = static.nn.fc(h, 3)
                    loss = paddle.nn.functional.cross_entropy(logits, y)
        opt_fn().minimize(loss)
    return main, startup, loss


def main():
    sched, mode = sys.argv[1], sys.argv[2]
    world = int(os.environ['WORLD_SIZE'])
    pp = 2 if mode == 'ppdp' else world
    dp = world // pp
    acc = 4
    amp_cfg = dict(init_loss_scaling=2.0 ** 24, use_dynamic_loss_scaling=True, incr_every_n_steps=1000,
                   decr_every_n_nan_or_inf=1, decr_ratio=2.0 ** -12)
    s = fleet.DistributedStrategy()
    if mode == 'ppamp':
        s.amp = True
        s.amp_configs = dict(amp_cfg)
    if mode == 'ppgm':
        s.gradient_merge = True
        s.gradient_merge_configs = {'k_steps': 2, 'avg': True}
    s.hybrid_configs = {'dp_degree': dp, 'mp_degree': 1, 'pp_degree': pp}
    s.pipeline = True
    s.pipeline_configs = {'accumulate_steps': acc, 'micro_batch_size': 2, 'schedule_mode': sched}
    V = 2 if sched == 'VPP' else 1
    if V > 1:
        s.pipeline_configs['vpp_degree'] = V
    builder = (lambda stages, fn: build_chain(stages * V, fn)) if V > 1 else build
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    rank = dist.get_rank()
    dp_rank = hcg.get_data_parallel_rank()
    paddle.enable_static()
    sgd = lambda: paddle.optimizer.SGD(learning_rate=0.2)  # noqa: E731
    main_p, startup, loss = builder(pp, lambda: fleet.distributed_optimizer(sgd()))
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    rng = np.random.RandomState(0)
    B = 8 * dp
    batches = []
    for _ in range(4 if mode == 'ppgm' else 3):
        xs = rng.randn(B, 6).astype('float32')
        batches.append((xs, (xs[:, :3].argmax(1)).reshape(-1, 1).astype('int64')))
    half = B // dp
    losses = []
    for xs, ys in batches:
        out = exe.run(main_p, feed={'x': xs[dp_rank * half:(dp_rank + 1) * half],
                                    'y': ys[dp_rank * half:(dp_rank + 1) * half]}, fetch_list=[loss])
        losses.append(float(np.asarray(out[0]).reshape(-1)[0]))
    if sched == 'ZBH1':
        from paddle.distributed.fleet.meta_parallel.zero_bubble_utils import WeightGradStore
        assert WeightGradStore.deferred > 0  # the stage's Linears ran as SplitBwLinear
    got = [p.numpy().copy() for p in main_p.all_parameters()]
    if mode == 'ppamp':
        import paddle.static.amp as samp
        ref_opt = lambda: samp.decorate(sgd(), level='O1', dtype='float16', **amp_cfg)  # noqa: E731
    else:
        ref_opt = sgd
    ref_main, ref_startup, ref_loss = builder(pp, ref_opt)
    ref_losses = []
    if mode == 'ppgm':  # the merged step == one full-batch step over both runs' samples
        batches = [(np.concatenate([batches[i][0], batches[i + 1][0]]),
                    np.concatenate([batches[i][1], batches[i + 1][1]])) for i in (0, 2)]
    for xs, ys in batches:
        # same micro-batch means as the pipeline: acc equal chunks of each dp shard, averaged
        out = exe.run(ref_main, feed={'x': xs, 'y': ys}, fetch_list=[ref_loss])
        ref_losses.append(float(np.asarray(out[0]).reshape(-1)[0]))
    # parameters in creation order: fc(x) w,b and skip w,b on stage 0, the middle fc on stage
    # min(1, pp-1), the head on the last stage; a rank owns (updates) its stage's parameters only
    st = [0, 0, 0, 0, min(1, pp - 1), min(1, pp - 1), pp - 1, pp - 1]
    if V > 1:  # chunk c of the chain lives on pipe rank c % pp
        st = [c % pp for c in range(pp * V) for _ in range(2)]
    me = hcg.get_stage_id()
    ref = [p.numpy() for p in ref_main.all_parameters()]
    assert len(got) == len(st) == len(ref), (len(got), len(ref))
    for a, b, s_ in zip(got, ref, st):
        if s_ == me:
            tol = 2e-3 if mode == 'ppamp' else 1e-4
            np.testing.assert_allclose(a, b, rtol=tol, atol=tol / 10)
    if mode == 'ppamp':
        pol = main_p.nodes[-1].target
        scale = pol._amp()._scale
        assert scale == 2.0 ** 12, scale  # the overflowing first step was skipped on every stage
    if dp == 1 and mode not in ('ppgm', 'ppamp'):
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-4, atol=1e-5)
    print(f"rank{rank} static pp {sched} {mode} OK", flush=True)


if __name__ == '__main__':
    main()
