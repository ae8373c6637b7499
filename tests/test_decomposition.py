"""paddle.decomposition: composite ops of a recorded static program replaced by primitives
(reference python/paddle/decomposition/decomp.py; rule set of paddle/fluid/primitive/composite/
composite.h).  Each case runs the program before and after ``decompose`` on the same feed."""
import numpy as np
import pytest

import paddle
from paddle.decomposition import decompose, register_decomp
from paddle.decomposition.decomp import op_name

F = paddle.nn.functional


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def _build(fn, shape=(None, 16)):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data('x', list(shape), 'float32')
        out = fn(x)
    return main, x, out


def _names(prog):
    return [op_name(n) for n in prog.nodes]


CASES = {
    'softmax': lambda x: F.softmax(x, -1),
    'log_softmax': lambda x: F.log_softmax(x, -1),
    'gelu': lambda x: F.gelu(x),
    'gelu_tanh': lambda x: F.gelu(x, approximate=True),
    'silu': lambda x: F.silu(x),
    'relu': lambda x: F.relu(x),
    'relu6': lambda x: F.relu6(x),
    'leaky_relu': lambda x: F.leaky_relu(x, 0.2),
    'elu': lambda x: F.elu(x, 0.7),
    'hardsigmoid': lambda x: F.hardsigmoid(x),
    'hardswish': lambda x: F.hardswish(x),
    'layer_norm': lambda x: paddle.nn.LayerNorm(16)(x),
    'mean_all': lambda x: paddle.mean(x),
    'mean_axis': lambda x: paddle.mean(x, axis=-1, keepdim=True),
    'linear': lambda x: paddle.nn.Linear(16, 8)(x),
    'square': lambda x: paddle.square(x),
    'clip': lambda x: paddle.clip(x, -0.5, 0.3),
    'flatten': lambda x: paddle.flatten(paddle.reshape(x, [-1, 4, 4]), 1),
    'unsqueeze': lambda x: paddle.unsqueeze(x, 1),
    'stack': lambda x: paddle.stack([x, x * 2], axis=1),
}


@pytest.mark.parametrize('case', sorted(CASES))
def test_decompose_matches(static_mode, case):
    paddle.seed(0)
    main, x, out = _build(CASES[case])
    exe = paddle.static.Executor()
    xv = np.random.RandomState(1).randn(5, 16).astype('float32')
    ref = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
    before = _names(main)
    assert any(before), before
    res = decompose(main, [out])
    assert res[0] is out
    assert not any(_names(main)), _names(main)  # every composite op is gone
    got = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)
    # dynamic batch: a different feed shape still runs (reduction counts re-specialised)
    xv2 = np.random.RandomState(2).randn(3, 16).astype('float32')
    got2 = exe.run(main, feed={'x': xv2}, fetch_list=[out])[0]
    paddle.disable_static()
    eager = CASES[case] if case not in ('layer_norm', 'linear') else None
    if eager is not None:
        np.testing.assert_allclose(got2, eager(paddle.to_tensor(xv2)).numpy(), rtol=1e-5, atol=1e-5)
    paddle.enable_static()


def test_white_black_lists_and_range(static_mode):
    main, x, out = _build(lambda x: F.gelu(F.softmax(x, -1)) + F.silu(x))
    decompose(main, [out], whitelist={'pd_op.softmax', 'pd_op.gelu'}, blacklist={'pd_op.gelu'})
    names = [n for n in _names(main) if n]
    assert names == ['pd_op.gelu', 'pd_op.silu'], names
    main, x, out = _build(lambda x: F.gelu(F.softmax(x, -1)) + F.silu(x))
    n0 = len(main.nodes)
    decompose(main, [out], start_index=1, end_index=2)  # only the gelu node
    names = [n for n in _names(main) if n]
    assert names == ['pd_op.softmax', 'pd_op.silu'], names
    assert len(main.nodes) > n0


def test_decomposed_program_trains(static_mode):
    """A decomposed MLP trains with the Executor: the captured parameters stay live (updates seen)."""
    paddle.seed(3)
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data('x', [None, 8], 'float32')
        y = paddle.static.data('y', [None, 1], 'float32')
        net = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.LayerNorm(16), paddle.nn.GELU(),
                                   paddle.nn.Linear(16, 1))
        loss = paddle.mean(paddle.square(net(x) - y))
        decompose(main, [loss])
        assert not any(_names(main))
        paddle.optimizer.SGD(0.1, parameters=net.parameters()).minimize(loss)
    exe = paddle.static.Executor()
    rs = np.random.RandomState(0)
    xv = rs.randn(32, 8).astype('float32')
    yv = (xv.sum(1, keepdims=True) * 0.3).astype('float32')
    losses = [float(exe.run(main, feed={'x': xv, 'y': yv}, fetch_list=[loss])[0]) for _ in range(30)]
    assert losses[-1] < 0.5 * losses[0], losses


def test_batch_norm_eval_and_custom_rule(static_mode):
    main, start = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, start):
        x = paddle.static.data('x', [None, 3, 4, 4], 'float32')
        bn = paddle.nn.BatchNorm2D(3)
        bn.eval()
        bn._mean.set_value(paddle.to_tensor([0.1, -0.2, 0.3]))
        bn._variance.set_value(paddle.to_tensor([1.5, 0.5, 2.0]))
        out = F.relu(bn(x))
    exe = paddle.static.Executor()
    xv = np.random.RandomState(0).randn(2, 3, 4, 4).astype('float32')
    ref = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
    decompose(main, [out])
    assert not any(_names(main))
    np.testing.assert_allclose(exe.run(main, feed={'x': xv}, fetch_list=[out])[0], ref, rtol=1e-5, atol=1e-5)

    calls = []

    @register_decomp('pd_op.silu')
    def my_silu(x, inplace=False):
        calls.append(1)
        return x * (1.0 / (1.0 + (-x).exp()))  # rules see the recorded (torch-level) arguments

    from paddle.decomposition import rules
    try:
        main, x, out = _build(lambda x: F.silu(x))
        decompose(main, [out])
        assert calls == [1]
    finally:
        register_decomp('pd_op.silu')(rules.silu)


def test_enable_prim_decomposes_on_run(static_mode):
    from paddle.incubate import autograd as A
    main, x, out = _build(lambda x: F.softmax(F.gelu(x), -1))
    exe = paddle.static.Executor()
    xv = np.random.RandomState(0).randn(4, 16).astype('float32')
    ref = exe.run(main, feed={'x': xv}, fetch_list=[out])[0]
    A.enable_prim()
    try:
        assert A.prim_enabled()
        main2, x2, out2 = _build(lambda x: F.softmax(F.gelu(x), -1))
        got = exe.run(main2, feed={'x': xv}, fetch_list=[out2])[0]
        assert not any(_names(main2))
    finally:
        A.disable_prim()
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
