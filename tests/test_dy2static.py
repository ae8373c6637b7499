"""dy2static: tensor-dependent Python control flow recorded as cond / while nodes.

Reference model: test/dygraph_to_static/test_ifelse.py, test_loop.py, test_logical.py,
test_return.py — a to_static function whose branches depend on tensor VALUES must give the
dygraph answer for every input after jit.save / jit.load (one saved program, both branches).
"""
import numpy as np
import pytest

import paddle
from paddle.static import InputSpec
from paddle.jit import dy2static


def _roundtrip(fn_or_layer, spec, tmp_path, name='m'):
    path = str(tmp_path / name)
    paddle.jit.save(fn_or_layer, path, input_spec=spec)
    return paddle.jit.load(path)


def _check(layer, loaded, xs):
    for x in xs:
        t = paddle.to_tensor(x)
        a = layer(t)
        b = loaded(t)
        a = a if isinstance(a, (list, tuple)) else [a]
        b = b if isinstance(b, (list, tuple)) else [b]
        for u, v in zip(a, b):
            np.testing.assert_allclose(u.numpy(), v.numpy(), rtol=1e-5, atol=1e-6)


class IfElseNet(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc = paddle.nn.Linear(4, 4)

    def forward(self, x):
        y = self.fc(x)
        if y.mean() > 0:
            z = y * 2
            only_true = z + 1
            z = only_true - 1
        else:
            z = y - 1
        return z


def test_if_else_both_branches(tmp_path):
    paddle.seed(0)
    net = IfElseNet()
    net.eval()
    tl = _roundtrip(net, [InputSpec([None, 4], 'float32')], tmp_path)
    xs = [np.full((2, 4), 5, 'float32'), np.full((3, 4), -5, 'float32')]
    means = [float(net(paddle.to_tensor(x)).mean()) for x in xs]
    assert (means[0] > 0) != (means[1] > 0)  # the two inputs really take different branches
    _check(net, tl, xs)


class EarlyReturn(paddle.nn.Layer):
    def forward(self, x):
        s = x.sum()
        if s > 10:
            return x * 3
        if s < -10:
            y = x - 100
            return y
        return x + 0.5


def test_early_return(tmp_path):
    net = EarlyReturn()
    tl = _roundtrip(net, [InputSpec([2, 4], 'float32')], tmp_path)
    _check(net, tl, [np.full((2, 4), v, 'float32') for v in (3.0, -3.0, 0.1)])


class WhileNet(paddle.nn.Layer):
    def forward(self, x, n):
        i = paddle.zeros([1], 'int64')
        acc = x
        while i < n:
            acc = acc * 2 + 1
            i = i + 1
        return acc, i


def test_while_tensor_bound(tmp_path):
    net = WhileNet()
    tl = _roundtrip(net, [InputSpec([3], 'float32'), InputSpec([1], 'int64')], tmp_path)
    x = np.arange(3, dtype='float32')
    for n in (0, 1, 4):
        a, ia = net(paddle.to_tensor(x), paddle.to_tensor(np.array([n], 'int64')))
        b, ib = tl(paddle.to_tensor(x), paddle.to_tensor(np.array([n], 'int64')))
        np.testing.assert_allclose(a.numpy(), b.numpy())
        assert int(ib.numpy()[0]) == n == int(ia.numpy()[0])


class ForRangeNet(paddle.nn.Layer):
    def forward(self, x, n):
        s = x * 0
        for k in range(n):
            s = s + x * k
        return s


def test_for_range_tensor_bound(tmp_path):
    net = ForRangeNet()
    tl = _roundtrip(net, [InputSpec([2], 'float32'), InputSpec([], 'int64')], tmp_path)
    x = np.array([1.0, 2.0], 'float32')
    for n in (0, 3, 5):
        nt = paddle.to_tensor(np.array(n, 'int64'))
        want = x * sum(range(n))
        np.testing.assert_allclose(tl(paddle.to_tensor(x), nt).numpy(), want, rtol=1e-6)
        np.testing.assert_allclose(net(paddle.to_tensor(x), nt).numpy(), want, rtol=1e-6)


class LogicNet(paddle.nn.Layer):
    def forward(self, x):
        a = x.mean()
        if a > 0 and x.max() < 10:
            y = x + 1
        elif not (a > -1) or x.min() > 100:
            y = x - 1
        else:
            y = x * 0
        z = y * 2 if y.sum() > 0 else y * 3
        return z


def test_logical_ops_and_ifexp(tmp_path):
    net = LogicNet()
    tl = _roundtrip(net, [InputSpec([4], 'float32')], tmp_path)
    _check(net, tl, [np.array(v, 'float32') for v in ([1, 2, 3, 4], [1, 2, 3, 40], [-5, -5, -5, -5],
                                                      [-0.5, -0.5, 0.2, 0.1])])


class Gate(paddle.nn.Layer):
    def forward(self, x):
        if x.mean() > 0:
            return paddle.nn.functional.relu(x)
        return -x


class Outer(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.gate = Gate()
        self.fc = paddle.nn.Linear(3, 3)

    def forward(self, x):
        return self.fc(self.gate(x))


def test_sublayer_forward_is_converted(tmp_path):
    paddle.seed(1)
    net = Outer()
    net.eval()
    tl = _roundtrip(net, [InputSpec([None, 3], 'float32')], tmp_path)
    _check(net, tl, [np.full((2, 3), 2, 'float32'), np.full((2, 3), -2, 'float32')])
    # the instance is left as it was (its forward is only swapped while recording)
    assert 'forward' not in net.gate.__dict__


def helper(x):
    if x.sum() > 0:
        out = x + 10
    else:
        out = x - 10
    return out


class CallsHelper(paddle.nn.Layer):
    def forward(self, x):
        return helper(x) * 2


def test_called_user_function_is_converted(tmp_path):
    net = CallsHelper()
    tl = _roundtrip(net, [InputSpec([2], 'float32')], tmp_path)
    _check(net, tl, [np.array([1, 2], 'float32'), np.array([-1, -2], 'float32')])


def test_python_predicates_stay_python():
    calls = []

    def f(x, flag=True):
        if flag:
            calls.append('t')
            y = x + 1
        else:
            calls.append('f')
            y = x - 1
        k = 0
        while k < 2:
            k += 1
        return y * k

    g = dy2static.convert_function(f)
    assert g is not f
    out = g(paddle.to_tensor([1.0]))
    assert calls == ['t'] and float(out) == 4.0
    # eager tensor predicates read the value, exactly like dygraph
    h = dy2static.convert_function(helper)
    assert float(h(paddle.to_tensor([1.0]))) == 11.0
    assert float(h(paddle.to_tensor([-1.0]))) == -11.0


def test_break_stays_python_and_not_to_static():
    def f(x):
        total = 0
        while True:
            total += 1
            if total > 3:
                break
        return x * total

    g = dy2static.convert_function(f)
    assert float(g(paddle.to_tensor(1.0))) == 4.0

    @paddle.jit.not_to_static
    def h(x):
        if x > 0:
            return x
        return -x
    assert dy2static.convert_function(h) is h


def test_static_function_code_shows_conversion():
    sf = paddle.jit.to_static(helper)
    assert 'convert_ifelse' in sf.code


def test_program_has_cond_node():
    net = IfElseNet()
    sf = paddle.jit.to_static(net.forward, input_spec=[InputSpec([None, 4], 'float32')])
    kinds = [n.kind for n in sf.concrete_program.main_program.nodes]
    assert 'cond' in kinds


def test_mismatched_python_values_raise():
    def f(x):
        if x.sum() > 0:
            mode = 'a'
        else:
            mode = 'b'
        return x, mode
    sf = paddle.jit.to_static(f, input_spec=[InputSpec([2], 'float32')])
    with pytest.raises(ValueError, match='different Python values'):
        sf.concrete_program
