"""paddle.distributed.passes over recorded static programs + fleet static collective training
(single-process parts; the 2-rank gloo parts are in test_distributed_cpu.py)."""
import numpy as np
import pytest

import paddle
import paddle.static as static


def _build(seed, opt_fn, clip=None):
    paddle.seed(seed)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 6], 'float32')
        y = static.data('y', [None, 1], 'int64')
        h = static.nn.fc(x, 12, activation='relu')
        logits = static.nn.fc(h, 3)
        loss = paddle.nn.functional.cross_entropy(logits, y)
        opt = opt_fn()
        if clip is not None:
            opt._grad_clip = clip
        opt.minimize(loss)
    return main, startup, loss


def _params(main):
    return [p.numpy().copy() for p in main.all_parameters()]


def _data(n=16, seed=0):
    rng = np.random.RandomState(seed)
    xs = rng.randn(n, 6).astype('float32')
    ys = (xs[:, :3].argmax(1)).reshape(-1, 1).astype('int64')
    return xs, ys


def test_new_pass_registry_and_manager_order(static_mode):
    from paddle.distributed.passes import new_pass, PassManager, PassContext
    with pytest.raises(AssertionError):
        new_pass('no_such_pass')
    gm = new_pass('auto_parallel_gradient_merge', {'k_steps': 2, 'avg': True})
    assert gm.get_attr('k_steps') == 2 and gm.name == 'auto_parallel_gradient_merge'
    amp1 = new_pass('auto_parallel_amp', {'dtype': 'bfloat16'})
    amp2 = new_pass('auto_parallel_fp16', {'dtype': 'bfloat16'})
    pm = PassManager([amp1, amp2, gm])
    assert isinstance(pm.context, PassContext)
    main, startup, _ = _build(1, lambda: paddle.optimizer.SGD(learning_rate=0.1))
    ctx = pm.apply([main], [startup])
    applied = [p.name for p in ctx.passes]
    # the two mixed-precision passes conflict: only one of them is applied
    assert sum(n in ('auto_parallel_amp', 'auto_parallel_fp16') for n in applied) == 1, applied
    assert 'auto_parallel_gradient_merge' in applied
    # a pass whose attributes make it inapplicable is dropped
    assert PassManager([new_pass('auto_parallel_gradient_merge', {'k_steps': 1})]).names == []


def test_gradient_merge_pass_matches_large_batch(static_mode):
    from paddle.distributed.passes import new_pass
    xs, ys = _data(16)
    sgd = lambda: paddle.optimizer.SGD(learning_rate=0.5)  # noqa: E731
    main, startup, loss = _build(3, sgd)
    p0 = _params(main)
    ctx = new_pass('auto_parallel_gradient_merge', {'k_steps': 2, 'avg': True}).apply([main], [startup])
    assert [p.name for p in ctx.passes] == ['auto_parallel_gradient_merge']
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    exe.run(main, feed={'x': xs[:8], 'y': ys[:8]}, fetch_list=[loss])
    for a, b in zip(_params(main), p0):  # no update after the first micro step
        np.testing.assert_array_equal(a, b)
    exe.run(main, feed={'x': xs[8:], 'y': ys[8:]}, fetch_list=[loss])
    merged = _params(main)
    ref_main, ref_startup, ref_loss = _build(3, sgd)
    exe.run(ref_startup)
    exe.run(ref_main, feed={'x': xs, 'y': ys}, fetch_list=[ref_loss])
    for a, b in zip(merged, _params(ref_main)):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def test_fleet_static_gradient_merge_strategy(static_mode):
    from paddle.distributed import fleet
    s = fleet.DistributedStrategy()
    s.gradient_merge = True
    s.gradient_merge_configs = {'k_steps': 2, 'avg': False}
    fleet.init(is_collective=True, strategy=s)
    xs, ys = _data(16, seed=1)
    sgd = lambda: paddle.optimizer.SGD(learning_rate=0.25)  # noqa: E731
    main, startup, loss = _build(5, lambda: fleet.distributed_optimizer(sgd()))
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    exe.run(main, feed={'x': xs[:8], 'y': ys[:8]}, fetch_list=[loss])
    exe.run(main, feed={'x': xs[8:], 'y': ys[8:]}, fetch_list=[loss])
    # avg=False: the merged gradient is the SUM of the two micro-batch means = 2 x the full-batch mean
    ref_main, ref_startup, ref_loss = _build(5, lambda: paddle.optimizer.SGD(learning_rate=0.5))
    exe.run(ref_startup)
    exe.run(ref_main, feed={'x': xs, 'y': ys}, fetch_list=[ref_loss])
    for a, b in zip(_params(main), _params(ref_main)):
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6)


def test_bf16_pass_matches_static_amp_decorate(static_mode):
    from paddle.distributed.passes import new_pass
    xs, ys = _data(16, seed=2)
    main, startup, loss = _build(9, lambda: paddle.optimizer.Adam(learning_rate=0.01))
    new_pass('auto_parallel_bf16', {}).apply([main], [startup])
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    la = [float(exe.run(main, feed={'x': xs, 'y': ys}, fetch_list=[loss])[0]) for _ in range(3)]
    ref_main, ref_startup, ref_loss = _build(
        9, lambda: paddle.static.amp.decorate(paddle.optimizer.Adam(learning_rate=0.01), level='O2',
                                              dtype='bfloat16', use_dynamic_loss_scaling=False))
    exe.run(ref_startup)
    lb = [float(exe.run(ref_main, feed={'x': xs, 'y': ys}, fetch_list=[ref_loss])[0]) for _ in range(3)]
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    assert str(main.all_parameters()[0].dtype).endswith('bfloat16')


def test_grad_clip_pass(static_mode):
    from paddle.distributed.passes import new_pass
    xs, ys = _data(16, seed=3)
    sgd = lambda: paddle.optimizer.SGD(learning_rate=1.0)  # noqa: E731
    main, startup, loss = _build(4, sgd)
    new_pass('auto_parallel_grad_clip', {'clip': paddle.nn.ClipGradByGlobalNorm(0.01)}).apply([main], [startup])
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    p0 = _params(main)
    exe.run(main, feed={'x': xs, 'y': ys}, fetch_list=[loss])
    delta = np.sqrt(sum(float(((a - b) ** 2).sum()) for a, b in zip(_params(main), p0)))
    assert delta <= 0.01 * 1.0001, delta  # lr 1 x a global norm clipped to 0.01
