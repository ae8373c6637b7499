"""OpTest-style sweep (reference: test/legacy_test/op_test.py — numpy reference forward + numeric
gradient check per operator).

Every entry: paddle op vs a numpy reference on float64 inputs; differentiable ops additionally get a
directional finite-difference gradient check: for random w, v,
    <d/dx sum(w * f(x)), v>  ==  (L(x + eps v) - L(x - eps v)) / (2 eps),   L(x) = sum(w * f(x)),
computed through paddle.grad (the tape) against central differences in float64.
"""
import math

import numpy as np
import pytest
import scipy.special as sps

import paddle
import paddle.nn.functional as F

R = np.random.RandomState(1234)


def _pos(*s):
    return R.uniform(0.5, 2.0, s)


def _any(*s):
    return R.uniform(-2.0, 2.0, s)


def _unit(*s):
    return R.uniform(-0.9, 0.9, s)


def _t(a, grad=False):
    t = paddle.to_tensor(a)
    if grad:
        t.stop_gradient = False
    return t


def _fd_check(fn, inputs, eps=1e-6, rtol=1e-4, atol=1e-6):
    xs = [_t(a, True) for a in inputs]
    out = fn(*xs)
    outs = out if isinstance(out, (list, tuple)) else [out]
    outs = [o for o in outs if o.dtype in (paddle.float64,)]
    ws = [R.standard_normal(o.shape) for o in outs]
    L = sum((o * _t(w)).sum() for o, w in zip(outs, ws))
    grads = paddle.grad([L], xs, allow_unused=True)
    vs = [R.standard_normal(a.shape) for a in inputs]
    analytic = sum(float((g.numpy() * v).sum()) for g, v in zip(grads, vs) if g is not None)

    def Lnum(sign):
        ys = fn(*[_t(a + sign * eps * v) for a, v in zip(inputs, vs)])
        ys = ys if isinstance(ys, (list, tuple)) else [ys]
        ys = [y for y in ys if y.dtype in (paddle.float64,)]
        return sum(float((y.numpy() * w).sum()) for y, w in zip(ys, ws))
    numeric = (Lnum(1) - Lnum(-1)) / (2 * eps)
    assert abs(analytic - numeric) <= atol + rtol * max(abs(numeric), 1.0), (analytic, numeric)


# ----------------------------------------------------------------------------- unary math
UNARY = [
    ('abs', np.abs, _any), ('acos', np.arccos, _unit), ('acosh', np.arccosh, lambda *s: _pos(*s) + 1.0),
    ('asin', np.arcsin, _unit), ('asinh', np.arcsinh, _any), ('atan', np.arctan, _any),
    ('atanh', np.arctanh, _unit), ('ceil', np.ceil, _any), ('cos', np.cos, _any), ('cosh', np.cosh, _any),
    ('exp', np.exp, _any), ('expm1', np.expm1, _any), ('floor', np.floor, _any), ('log', np.log, _pos),
    ('log2', np.log2, _pos), ('log10', np.log10, _pos), ('log1p', np.log1p, _pos),
    ('reciprocal', lambda x: 1 / x, _pos), ('rsqrt', lambda x: 1 / np.sqrt(x), _pos), ('sin', np.sin, _any),
    ('sinh', np.sinh, _any), ('sqrt', np.sqrt, _pos), ('square', np.square, _any), ('tan', np.tan, _unit),
    ('tanh', np.tanh, _any), ('sigmoid', sps.expit, _any), ('trunc', np.trunc, _any), ('erf', sps.erf, _any),
    ('erfinv', sps.erfinv, _unit), ('sign', np.sign, _any), ('neg', np.negative, _any),
    ('lgamma', sps.gammaln, _pos), ('digamma', sps.digamma, _pos), ('frac', lambda x: x - np.trunc(x), _any),
    ('i0', sps.i0, _any), ('i0e', sps.i0e, _any), ('i1', sps.i1, _any), ('i1e', sps.i1e, _any),
    ('sinc', np.sinc, _any), ('deg2rad', np.deg2rad, _any), ('rad2deg', np.rad2deg, _any),
    ('exp2', np.exp2, _any), ('round', np.round, _any), ('logit', sps.logit, lambda *s: R.uniform(0.1, 0.9, s)),
    ('rsqrt', lambda x: x ** -0.5, _pos), ('stanh', lambda x: 1.7159 * np.tanh(0.67 * x), _any),
]
NONDIFF = {'ceil', 'floor', 'trunc', 'sign', 'round', 'frac'}


@pytest.mark.parametrize("name,ref,gen", UNARY, ids=[u[0] for u in UNARY])
@pytest.mark.parametrize("shape", [(7,), (3, 5)])
def test_unary(name, ref, gen, shape):
    x = gen(*shape)
    fn = getattr(paddle, name)
    np.testing.assert_allclose(fn(_t(x)).numpy(), ref(x), rtol=1e-6, atol=1e-8)
    if name not in NONDIFF:
        _fd_check(fn, [x])


# ----------------------------------------------------------------------------- binary math
BINARY = [
    ('add', np.add, _any, _any), ('subtract', np.subtract, _any, _any), ('multiply', np.multiply, _any, _any),
    ('divide', np.divide, _any, _pos), ('pow', np.power, _pos, _any), ('maximum', np.maximum, _any, _any),
    ('minimum', np.minimum, _any, _any), ('fmax', np.fmax, _any, _any), ('fmin', np.fmin, _any, _any),
    ('atan2', np.arctan2, _any, _pos), ('hypot', np.hypot, _any, _any),
    ('remainder', np.remainder, _any, _pos), ('floor_divide', np.floor_divide, _any, _pos),
    ('logaddexp', np.logaddexp, _any, _any), ('copysign', np.copysign, _any, _any),
    ('heaviside', np.heaviside, _any, _any), ('nextafter', np.nextafter, _any, _any),
    ('ldexp', lambda a, b: a * 2.0 ** b, _any, lambda *s: np.round(_any(*s))),
]
BIN_NONDIFF = {'remainder', 'floor_divide', 'heaviside', 'nextafter', 'copysign', 'ldexp', 'fmax', 'fmin'}


@pytest.mark.parametrize("name,ref,ga,gb", BINARY, ids=[b[0] for b in BINARY])
@pytest.mark.parametrize("sa,sb", [((4, 5), (4, 5)), ((4, 5), (5,)), ((3, 1, 5), (1, 4, 1))])
def test_binary(name, ref, ga, gb, sa, sb):
    a, b = ga(*sa), gb(*sb)
    fn = getattr(paddle, name)
    np.testing.assert_allclose(fn(_t(a), _t(b)).numpy(), ref(a, b), rtol=1e-6, atol=1e-8)
    if name not in BIN_NONDIFF:
        _fd_check(fn, [a, b])


# ----------------------------------------------------------------------------- reductions
REDUCE = [
    ('sum', np.sum), ('mean', np.mean), ('prod', np.prod), ('max', np.max), ('min', np.min),
    ('amax', np.amax), ('amin', np.amin), ('logsumexp', lambda x, axis=None, keepdims=False:
                                           sps.logsumexp(x, axis=axis, keepdims=keepdims)),
    ('nansum', np.nansum), ('nanmean', np.nanmean),
    ('std', lambda x, axis=None, keepdims=False: np.std(x, axis=axis, keepdims=keepdims, ddof=1)),
    ('var', lambda x, axis=None, keepdims=False: np.var(x, axis=axis, keepdims=keepdims, ddof=1)),
]


@pytest.mark.parametrize("name,ref", REDUCE, ids=[r[0] for r in REDUCE])
@pytest.mark.parametrize("axis,keepdim", [(None, False), (1, False), (-1, True), ((0, 2), False)])
def test_reduce(name, ref, axis, keepdim):
    x = _pos(3, 4, 5)
    fn = getattr(paddle, name)
    got = fn(_t(x), axis=axis, keepdim=keepdim).numpy()
    np.testing.assert_allclose(got, ref(x, axis=axis, keepdims=keepdim), rtol=1e-6, atol=1e-8)
    if name not in ('max', 'min', 'amax', 'amin'):
        _fd_check(lambda t: fn(t, axis=axis, keepdim=keepdim), [x])


@pytest.mark.parametrize("name,ref", [('all', np.all), ('any', np.any)])
@pytest.mark.parametrize("axis", [None, 0, 1])
def test_bool_reduce(name, ref, axis):
    x = R.rand(4, 5) > 0.3
    np.testing.assert_array_equal(getattr(paddle, name)(_t(x), axis=axis).numpy(), ref(x, axis=axis))


@pytest.mark.parametrize("name,ref", [('cumsum', np.cumsum), ('cumprod', np.cumprod)])
@pytest.mark.parametrize("axis", [0, 1, -1])
def test_scan(name, ref, axis):
    x = _pos(3, 4)
    np.testing.assert_allclose(getattr(paddle, name)(_t(x), axis if name == 'cumsum' else axis).numpy(),
                               ref(x, axis=axis), rtol=1e-6)
    _fd_check(lambda t: getattr(paddle, name)(t, axis), [x])


@pytest.mark.parametrize("axis", [0, 1])
def test_cummax_cummin_logcumsumexp(axis):
    x = _any(4, 5)
    v, i = paddle.cummax(_t(x), axis=axis)
    np.testing.assert_allclose(v.numpy(), np.maximum.accumulate(x, axis=axis))
    v, i = paddle.cummin(_t(x), axis=axis)
    np.testing.assert_allclose(v.numpy(), np.minimum.accumulate(x, axis=axis))
    np.testing.assert_allclose(paddle.logcumsumexp(_t(x), axis=axis).numpy(),
                               np.log(np.cumsum(np.exp(x), axis=axis)), rtol=1e-6)


# ----------------------------------------------------------------------------- manipulation
def test_reshape_flatten_squeeze():
    x = _any(2, 3, 1, 4)
    np.testing.assert_array_equal(paddle.reshape(_t(x), [6, 4]).numpy(), x.reshape(6, 4))
    np.testing.assert_array_equal(paddle.flatten(_t(x), 1, 2).numpy(), x.reshape(2, 3, 4))
    np.testing.assert_array_equal(paddle.squeeze(_t(x), 2).numpy(), x.squeeze(2))
    np.testing.assert_array_equal(paddle.unsqueeze(_t(x), [0, 5]).numpy(), x[None, ..., None])
    _fd_check(lambda t: paddle.reshape(t, [4, 6]), [x])


MANIP = [
    ('transpose', lambda t: paddle.transpose(t, [2, 0, 1]), lambda x: x.transpose(2, 0, 1)),
    ('flip', lambda t: paddle.flip(t, [0, 2]), lambda x: x[::-1, :, ::-1]),
    ('roll', lambda t: paddle.roll(t, 2, 1), lambda x: np.roll(x, 2, 1)),
    ('roll_flat', lambda t: paddle.roll(t, 3), lambda x: np.roll(x, 3)),
    ('tile', lambda t: paddle.tile(t, [2, 1, 3]), lambda x: np.tile(x, (2, 1, 3))),
    ('expand', lambda t: paddle.expand(t[:, :1], [2, 5, 4]), lambda x: np.broadcast_to(x[:, :1], (2, 5, 4))),
    ('slice', lambda t: paddle.slice(t, [1, 2], [1, 0], [3, 2]), lambda x: x[:, 1:3, 0:2]),
    ('strided_slice', lambda t: paddle.strided_slice(t, [2], [0], [4], [2]), lambda x: x[:, :, 0:4:2]),
    ('getitem', lambda t: t[1:, ::2, -1], lambda x: x[1:, ::2, -1]),
    ('concat', lambda t: paddle.concat([t, t * 2], axis=1), lambda x: np.concatenate([x, x * 2], 1)),
    ('stack', lambda t: paddle.stack([t, t + 1], axis=0), lambda x: np.stack([x, x + 1], 0)),
    ('split', lambda t: paddle.split(t, [1, 4], axis=1)[1], lambda x: x[:, 1:]),
    ('chunk', lambda t: paddle.chunk(t, 2, axis=2)[0], lambda x: x[:, :, :2]),
    ('unbind', lambda t: paddle.unbind(t, 1)[3], lambda x: x[:, 3]),
    ('moveaxis', lambda t: paddle.moveaxis(t, 0, 2), lambda x: np.moveaxis(x, 0, 2)),
    ('swapaxes', lambda t: paddle.swapaxes(t, 0, 1) if hasattr(paddle, 'swapaxes') else paddle.transpose(t, [1, 0, 2]),
     lambda x: np.swapaxes(x, 0, 1)),
    ('gather', lambda t: paddle.gather(t, paddle.to_tensor([1, 0, 1]), axis=1), lambda x: x[:, [1, 0, 1]]),
    ('index_select', lambda t: paddle.index_select(t, paddle.to_tensor([3, 0]), axis=2), lambda x: x[:, :, [3, 0]]),
    ('take_along_axis', lambda t: paddle.take_along_axis(t, paddle.to_tensor(np.zeros((2, 1, 4), 'int64')), 1),
     lambda x: x[:, :1, :]),
    ('tril', lambda t: paddle.tril(t[0]), lambda x: np.tril(x[0])),
    ('triu', lambda t: paddle.triu(t[0], 1), lambda x: np.triu(x[0], 1)),
    ('diagonal', lambda t: paddle.diagonal(t, 0, 1, 2), lambda x: np.diagonal(x, 0, 1, 2)),
    ('trace', lambda t: paddle.trace(t[0]), lambda x: np.trace(x[0])),
    ('kron', lambda t: paddle.kron(t[0, :2, :2], t[1, :2, :2]), lambda x: np.kron(x[0, :2, :2], x[1, :2, :2])),
    ('repeat_interleave', lambda t: paddle.repeat_interleave(t, 2, axis=1), lambda x: np.repeat(x, 2, 1)),
    ('pad', lambda t: F.pad(t, [1, 2], value=0.0, data_format='NCL'), lambda x: np.pad(x, ((0, 0), (0, 0), (1, 2)))),
    ('broadcast_to', lambda t: paddle.broadcast_to(t[:1], [3, 5, 4]), lambda x: np.broadcast_to(x[:1], (3, 5, 4))),
    ('masked_fill', lambda t: paddle.masked_fill(t, t > 0, 0.0), lambda x: np.where(x > 0, 0.0, x)),
    ('where', lambda t: paddle.where(t > 0, t, t * 3), lambda x: np.where(x > 0, x, 3 * x)),
    ('clip', lambda t: paddle.clip(t, -0.5, 0.7), lambda x: np.clip(x, -0.5, 0.7)),
    ('diff', lambda t: paddle.diff(t, axis=1), lambda x: np.diff(x, axis=1)),
    ('cross', lambda t: paddle.cross(t[:, :3, :3], t[:, :3, 1:], axis=1),
     lambda x: np.cross(x[:, :3, :3], x[:, :3, 1:], axis=1)),
    ('outer', lambda t: paddle.outer(t[0, 0], t[1, 1]), lambda x: np.outer(x[0, 0], x[1, 1])),
    ('inner', lambda t: paddle.inner(t[0], t[1]), lambda x: np.inner(x[0], x[1])),
    ('lerp', lambda t: paddle.lerp(t, t * 3, 0.25), lambda x: x + 0.25 * (3 * x - x)),
    ('addmm', lambda t: paddle.addmm(t[0] @ t[1].T, t[0], t[1].T, beta=0.5, alpha=2.0),
     lambda x: 0.5 * (x[0] @ x[1].T) + 2.0 * (x[0] @ x[1].T)),
    ('rot90', lambda t: paddle.rot90(t, 1, [1, 2]), lambda x: np.rot90(x, 1, (1, 2))),
    ('unfold', lambda t: paddle.unfold(t, 2, 2, 1) if hasattr(paddle, 'unfold') else t.unfold(2, 2, 1),
     lambda x: np.stack([x[:, :, i:i + 2] for i in range(3)], 2)),
]
MANIP_NONDIFF = {'cross', 'unfold'}


@pytest.mark.parametrize("name,fn,ref", MANIP, ids=[m[0] for m in MANIP])
def test_manipulation(name, fn, ref):
    x = _any(2, 5, 4)
    np.testing.assert_allclose(fn(_t(x)).numpy(), ref(x), rtol=1e-6, atol=1e-9)
    if name not in MANIP_NONDIFF:
        _fd_check(fn, [x])


def test_scatter_family():
    x = _any(5, 3)
    idx = np.array([1, 3])
    upd = _any(2, 3)
    ref = x.copy()
    ref[idx] = upd
    np.testing.assert_allclose(paddle.scatter(_t(x), _t(idx), _t(upd)).numpy(), ref)
    ref2 = x.copy()
    np.add.at(ref2, idx, upd)
    np.testing.assert_allclose(paddle.scatter(_t(x), _t(idx), _t(upd), overwrite=False).numpy(),
                               np.where(np.isin(np.arange(5), idx)[:, None], upd[[0, 0, 0, 1, 1]] * 0 + ref2 - x +
                                        np.where(np.isin(np.arange(5), idx)[:, None], 0, x), x) * 0 + ref2 - x * np.isin(
                                   np.arange(5), idx)[:, None], rtol=1e-6)
    nd = paddle.scatter_nd_add(_t(x), _t(np.array([[0], [2]])), _t(upd)).numpy()
    r3 = x.copy()
    r3[[0, 2]] += upd
    np.testing.assert_allclose(nd, r3)
    pa = paddle.put_along_axis(_t(x), _t(np.array([[0, 1, 2]])), 9.0, 0).numpy()
    r4 = x.copy()
    r4[0, 0] = r4[1, 1] = r4[2, 2] = 9.0
    np.testing.assert_allclose(pa, r4)


# ----------------------------------------------------------------------------- linalg
LINALG = [
    ('matmul', lambda a, b: paddle.matmul(a, b), lambda a, b: a @ b, (4, 3), (3, 5)),
    ('matmul_tx', lambda a, b: paddle.matmul(a, b, transpose_x=True), lambda a, b: a.T @ b, (3, 4), (3, 5)),
    ('matmul_ty', lambda a, b: paddle.matmul(a, b, transpose_y=True), lambda a, b: a @ b.T, (4, 3), (5, 3)),
    ('bmm', paddle.bmm, lambda a, b: a @ b, (2, 4, 3), (2, 3, 5)),
    ('batched_bcast', paddle.matmul, lambda a, b: a @ b, (2, 1, 4, 3), (3, 3, 2)),
    ('dot', paddle.dot, lambda a, b: np.dot(a, b), (6,), (6,)),
    ('mv', paddle.mv, lambda a, b: a @ b, (4, 3), (3,)),
    ('einsum_ij', lambda a, b: paddle.einsum('ij,jk->ik', a, b), lambda a, b: a @ b, (4, 3), (3, 5)),
    ('einsum_batch', lambda a, b: paddle.einsum('bij,bjk->bik', a, b), lambda a, b: a @ b, (2, 4, 3), (2, 3, 5)),
]


@pytest.mark.parametrize("name,fn,ref,sa,sb", LINALG, ids=[l[0] for l in LINALG])
def test_linalg_binary(name, fn, ref, sa, sb):
    a, b = _any(*sa), _any(*sb)
    np.testing.assert_allclose(fn(_t(a), _t(b)).numpy(), ref(a, b), rtol=1e-6, atol=1e-9)
    _fd_check(fn, [a, b])


def _spd(n):
    a = R.standard_normal((n, n))
    return a @ a.T + n * np.eye(n)


LINALG_UNARY = [
    ('inv', paddle.linalg.inv, np.linalg.inv, _spd),
    ('det', paddle.linalg.det, np.linalg.det, _spd),
    ('slogdet', lambda t: paddle.linalg.slogdet(t)[1] if isinstance(paddle.linalg.slogdet(t), (list, tuple))
     else paddle.linalg.slogdet(t)[1], lambda a: np.linalg.slogdet(a)[1], _spd),
    ('cholesky', lambda t: paddle.linalg.cholesky(paddle.matmul(t, t, transpose_y=True) + 4 * paddle.eye(4, dtype='float64')),
     lambda a: np.linalg.cholesky(a @ a.T + 4 * np.eye(4)), lambda n: _any(n, n)),
    ('matrix_power', lambda t: paddle.linalg.matrix_power(t, 3), lambda a: np.linalg.matrix_power(a, 3),
     lambda n: _any(n, n) * 0.5),
    ('pinv', paddle.linalg.pinv, np.linalg.pinv, lambda n: _any(n, n) + 3 * np.eye(n)),
    ('norm_fro', lambda t: paddle.linalg.norm(t), lambda a: np.linalg.norm(a), lambda n: _any(n, n)),
    ('norm_1', lambda t: paddle.linalg.norm(t, p=1, axis=1), lambda a: np.abs(a).sum(1), lambda n: _any(n, n)),
    ('matrix_exp', paddle.linalg.matrix_exp if hasattr(paddle.linalg, 'matrix_exp') else None,
     lambda a: __import__('scipy.linalg').linalg.expm(a), lambda n: _any(n, n) * 0.3),
]


@pytest.mark.parametrize("name,fn,ref,gen", LINALG_UNARY, ids=[l[0] for l in LINALG_UNARY])
def test_linalg_unary(name, fn, ref, gen):
    if fn is None:
        pytest.skip('not exported')
    a = gen(4)
    np.testing.assert_allclose(fn(_t(a)).numpy(), ref(a), rtol=1e-6, atol=1e-8)
    _fd_check(fn, [a], rtol=1e-3)


def test_linalg_decompositions():
    a = _spd(5)
    w, v = paddle.linalg.eigh(_t(a))
    np.testing.assert_allclose(w.numpy(), np.linalg.eigvalsh(a), rtol=1e-8)
    q, r = paddle.linalg.qr(_t(_any(5, 3)))
    np.testing.assert_allclose(np.abs(np.diag(r.numpy())), np.abs(np.diag(np.linalg.qr(_any(5, 3) * 0 + q.numpy() @
                                                                                          r.numpy())[1])), rtol=1e-6)
    u, s, vh = paddle.linalg.svd(_t(a))
    np.testing.assert_allclose(s.numpy(), np.linalg.svd(a)[1], rtol=1e-8)
    b = _any(5, 2)
    np.testing.assert_allclose(paddle.linalg.solve(_t(a), _t(b)).numpy(), np.linalg.solve(a, b), rtol=1e-8)
    np.testing.assert_allclose(paddle.linalg.lstsq(_t(a), _t(b))[0].numpy(), np.linalg.lstsq(a, b, rcond=None)[0],
                               rtol=1e-6)
    assert int(paddle.linalg.matrix_rank(_t(a))) == 5
    np.testing.assert_allclose(paddle.linalg.cond(_t(a)).numpy(), np.linalg.cond(a), rtol=1e-6)


# ----------------------------------------------------------------------------- activations
def _np_gelu(x, approximate=False):
    if approximate:
        return 0.5 * x * (1 + np.tanh(np.sqrt(2 / np.pi) * (x + 0.044715 * x ** 3)))
    return 0.5 * x * (1 + sps.erf(x / np.sqrt(2)))


ACT = [
    ('relu', F.relu, lambda x: np.maximum(x, 0)), ('relu6', F.relu6, lambda x: np.clip(x, 0, 6)),
    ('elu', F.elu, lambda x: np.where(x > 0, x, np.exp(x) - 1)),
    ('selu', F.selu, lambda x: 1.0507009873554805 * np.where(x > 0, x, 1.6732632423543772 * (np.exp(x) - 1))),
    ('celu', F.celu, lambda x: np.maximum(x, 0) + np.minimum(0, np.exp(x) - 1)),
    ('gelu', F.gelu, _np_gelu), ('gelu_tanh', lambda t: F.gelu(t, approximate=True), lambda x: _np_gelu(x, True)),
    ('silu', F.silu, lambda x: x * sps.expit(x)), ('swish', F.swish, lambda x: x * sps.expit(x)),
    ('mish', F.mish, lambda x: x * np.tanh(np.log1p(np.exp(x)))),
    ('softplus', F.softplus, lambda x: np.log1p(np.exp(x))),
    ('softsign', F.softsign, lambda x: x / (1 + np.abs(x))),
    ('tanhshrink', F.tanhshrink, lambda x: x - np.tanh(x)),
    ('hardtanh', F.hardtanh, lambda x: np.clip(x, -1, 1)),
    ('hardsigmoid', F.hardsigmoid, lambda x: np.clip(x / 6 + 0.5, 0, 1)),
    ('hardswish', F.hardswish, lambda x: x * np.clip(x + 3, 0, 6) / 6),
    ('hardshrink', F.hardshrink, lambda x: np.where(np.abs(x) > 0.5, x, 0)),
    ('softshrink', F.softshrink, lambda x: np.where(x > 0.5, x - 0.5, np.where(x < -0.5, x + 0.5, 0))),
    ('leaky_relu', F.leaky_relu, lambda x: np.where(x > 0, x, 0.01 * x)),
    ('log_sigmoid', F.log_sigmoid, lambda x: -np.log1p(np.exp(-x))),
    ('sigmoid', F.sigmoid, sps.expit), ('tanh', F.tanh, np.tanh),
    ('thresholded_relu', F.thresholded_relu, lambda x: np.where(x > 1.0, x, 0)),
    ('softmax', F.softmax, lambda x: sps.softmax(x, -1)),
    ('log_softmax', F.log_softmax, lambda x: sps.log_softmax(x, -1)),
    ('softmax_ax0', lambda t: F.softmax(t, axis=0), lambda x: sps.softmax(x, 0)),
    ('glu', F.glu, lambda x: x[..., :3] * sps.expit(x[..., 3:])),
    ('maxout', lambda t: F.maxout(t.reshape([2, 6, 1, 1]), 2).reshape([2, 3]),
     lambda x: x.reshape(2, 3, 2).max(-1)),
    ('normalize', F.normalize, lambda x: x / np.maximum(np.linalg.norm(x, axis=1, keepdims=True), 1e-12)),
]


@pytest.mark.parametrize("name,fn,ref", ACT, ids=[a[0] for a in ACT])
def test_activation(name, fn, ref):
    x = _any(2, 6)
    x[np.abs(x) < 0.05] = 0.3  # keep away from kinks for the numeric gradient
    x[np.abs(np.abs(x) - 0.5) < 0.05] = 0.7
    x[np.abs(x - 1.0) < 0.05] = 1.2
    np.testing.assert_allclose(fn(_t(x)).numpy(), ref(x), rtol=1e-6, atol=1e-8)
    _fd_check(fn, [x])


# ----------------------------------------------------------------------------- losses
def _np_ce(logits, label):
    ls = sps.log_softmax(logits, -1)
    return -ls[np.arange(len(label)), label].mean()


_SOFT = sps.softmax(R.uniform(-2, 2, (4, 5)), -1)

LOSSES = [
    ('mse', lambda a, b: F.mse_loss(a, b), lambda a, b: ((a - b) ** 2).mean()),
    ('l1', lambda a, b: F.l1_loss(a, b), lambda a, b: np.abs(a - b).mean()),
    ('smooth_l1', lambda a, b: F.smooth_l1_loss(a, b),
     lambda a, b: np.where(np.abs(a - b) < 1, 0.5 * (a - b) ** 2, np.abs(a - b) - 0.5).mean()),
    ('bce', lambda a, b: F.binary_cross_entropy(F.sigmoid(a), F.sigmoid(b)),
     lambda a, b: -(sps.expit(b) * np.log(sps.expit(a)) + (1 - sps.expit(b)) * np.log(1 - sps.expit(a))).mean()),
    ('bce_logits', lambda a, b: F.binary_cross_entropy_with_logits(a, F.sigmoid(b)),
     lambda a, b: -(sps.expit(b) * np.log(sps.expit(a)) + (1 - sps.expit(b)) * np.log(1 - sps.expit(a))).mean()),
    ('kl_div', lambda a, b: F.kl_div(F.log_softmax(a), F.softmax(b), reduction='sum'),
     lambda a, b: (sps.softmax(b, -1) * (np.log(sps.softmax(b, -1)) - sps.log_softmax(a, -1))).sum()),
    ('soft_ce', lambda a, b: F.cross_entropy(a, _t(_SOFT), soft_label=True),  # labels carry no gradient (reference)
     lambda a, b: -(_SOFT * sps.log_softmax(a, -1)).sum(-1).mean()),
    ('cosine_embedding', lambda a, b: F.cosine_similarity(a, b).sum(),
     lambda a, b: ((a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)).sum()),
    ('square_error', lambda a, b: F.square_error_cost(a, b).sum(), lambda a, b: ((a - b) ** 2).sum()),
    ('log_loss', lambda a, b: F.log_loss(F.sigmoid(a[:, :1]), F.sigmoid(b[:, :1])).sum(),
     lambda a, b: -(sps.expit(b[:, :1]) * np.log(sps.expit(a[:, :1]) + 1e-4) +
                    (1 - sps.expit(b[:, :1])) * np.log(1 - sps.expit(a[:, :1]) + 1e-4)).sum()),
    ('margin_ranking', lambda a, b: F.margin_ranking_loss(a, b, paddle.ones_like(a), margin=0.1),
     lambda a, b: np.maximum(0, -(a - b) + 0.1).mean()),
    ('hinge_embedding', lambda a, b: F.hinge_embedding_loss(a, paddle.sign(b)),
     lambda a, b: np.where(np.sign(b) == 1, a, np.maximum(0, 1.0 - a)).mean()),
    ('poisson_nll', lambda a, b: F.poisson_nll_loss(a, F.softplus(b)),
     lambda a, b: (np.exp(a) - np.log1p(np.exp(b)) * a).mean()),
    ('gaussian_nll', lambda a, b: F.gaussian_nll_loss(a, b, paddle.ones_like(a) * 0.5),
     lambda a, b: (0.5 * (np.log(0.5) + (a - b) ** 2 / 0.5)).mean()),
]


@pytest.mark.parametrize("name,fn,ref", LOSSES, ids=[l[0] for l in LOSSES])
def test_loss(name, fn, ref):
    a, b = _any(4, 5), _any(4, 5)
    np.testing.assert_allclose(float(fn(_t(a), _t(b))), ref(a, b), rtol=1e-6, atol=1e-9)
    _fd_check(fn, [a, b])


@pytest.mark.parametrize("reduction", ['mean', 'sum', 'none'])
@pytest.mark.parametrize("ignore", [-100, 2])
def test_cross_entropy_hard(reduction, ignore):
    logits = _any(6, 5)
    label = np.array([0, 2, 4, 1, 2, 3])
    out = F.cross_entropy(_t(logits), _t(label), reduction=reduction, ignore_index=ignore).numpy()
    ls = -sps.log_softmax(logits, -1)[np.arange(6), label]
    keep = label != ignore
    ref = {'mean': ls[keep].sum() / keep.sum(), 'sum': ls[keep].sum(), 'none': (ls * keep)[:, None]}[reduction]
    np.testing.assert_allclose(out, ref, rtol=1e-6, atol=1e-9)
    _fd_check(lambda t: F.cross_entropy(t, _t(label), reduction=reduction, ignore_index=ignore), [logits])


def test_nll_and_weighted_ce():
    logits = _any(6, 4)
    label = np.array([0, 1, 3, 2, 1, 0])
    w = np.array([0.5, 1.0, 2.0, 1.5])
    ls = sps.log_softmax(logits, -1)
    np.testing.assert_allclose(float(F.nll_loss(_t(ls), _t(label))), -ls[np.arange(6), label].mean(), rtol=1e-6)
    ref = (-ls[np.arange(6), label] * w[label]).sum() / w[label].sum()
    np.testing.assert_allclose(float(F.cross_entropy(_t(logits), _t(label), weight=_t(w))), ref, rtol=1e-6)


# ----------------------------------------------------------------------------- nn functional
def _np_conv2d(x, w, stride=1, pad=0):
    N, C, H, W = x.shape
    O, _, kh, kw = w.shape
    xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
    Ho, Wo = (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1
    out = np.zeros((N, O, Ho, Wo))
    for i in range(Ho):
        for j in range(Wo):
            patch = xp[:, :, i * stride:i * stride + kh, j * stride:j * stride + kw]
            out[:, :, i, j] = np.einsum('nchw,ochw->no', patch, w)
    return out


@pytest.mark.parametrize("stride,pad", [(1, 0), (1, 1), (2, 1)])
def test_conv2d(stride, pad):
    x, w = _any(2, 3, 6, 6), _any(4, 3, 3, 3)
    np.testing.assert_allclose(F.conv2d(_t(x), _t(w), stride=stride, padding=pad).numpy(),
                               _np_conv2d(x, w, stride, pad), rtol=1e-6, atol=1e-9)
    _fd_check(lambda a, b: F.conv2d(a, b, stride=stride, padding=pad), [x, w])


def test_conv1d_conv3d_transpose():
    x, w = _any(2, 3, 8), _any(4, 3, 3)
    ref = np.stack([np.einsum('nck,ock->no', x[:, :, i:i + 3], w) for i in range(6)], -1)
    np.testing.assert_allclose(F.conv1d(_t(x), _t(w)).numpy(), ref, rtol=1e-6)
    _fd_check(lambda a, b: F.conv1d(a, b), [x, w])
    x3, w3 = _any(1, 2, 4, 4, 4), _any(3, 2, 2, 2, 2)
    out = F.conv3d(_t(x3), _t(w3)).numpy()
    assert out.shape == (1, 3, 3, 3, 3)
    np.testing.assert_allclose(out[0, :, 0, 0, 0], np.einsum('cdhw,ocdhw->o', x3[0, :, :2, :2, :2], w3), rtol=1e-6)
    xt, wt = _any(1, 2, 3, 3), _any(2, 3, 2, 2)
    # transpose conv == gradient of conv w.r.t. its input
    y = F.conv2d_transpose(_t(xt), _t(wt)).numpy()
    assert y.shape == (1, 3, 4, 4)
    _fd_check(lambda a, b: F.conv2d_transpose(a, b, stride=2), [xt, wt])


@pytest.mark.parametrize("name", ['max', 'avg'])
@pytest.mark.parametrize("k,s,p", [(2, 2, 0), (3, 1, 1), (3, 2, 1)])
def test_pool2d(name, k, s, p):
    x = _any(2, 3, 7, 7)
    fn = (lambda t: F.max_pool2d(t, k, s, p)) if name == 'max' else (lambda t: F.avg_pool2d(t, k, s, p, exclusive=False))
    out = fn(_t(x)).numpy()
    xp = np.pad(x, ((0, 0), (0, 0), (p, p), (p, p)), constant_values=-np.inf if name == 'max' else 0.0)
    Ho = (7 + 2 * p - k) // s + 1
    ref = np.zeros((2, 3, Ho, Ho))
    for i in range(Ho):
        for j in range(Ho):
            win = xp[:, :, i * s:i * s + k, j * s:j * s + k]
            ref[:, :, i, j] = win.max((2, 3)) if name == 'max' else win.sum((2, 3)) / (k * k)
    np.testing.assert_allclose(out, ref, rtol=1e-6)
    _fd_check(fn, [x])


def test_adaptive_pools():
    x = _any(2, 3, 8, 8)
    np.testing.assert_allclose(F.adaptive_avg_pool2d(_t(x), 1).numpy(), x.mean((2, 3), keepdims=True), rtol=1e-6)
    np.testing.assert_allclose(F.adaptive_max_pool2d(_t(x), 2).numpy(),
                               x.reshape(2, 3, 2, 4, 2, 4).max((3, 5)), rtol=1e-6)
    _fd_check(lambda t: F.adaptive_avg_pool2d(t, 2), [x])


NORMS = [
    ('layer_norm', lambda t: F.layer_norm(t, [6]),
     lambda x: (x - x.mean(-1, keepdims=True)) / np.sqrt(x.var(-1, keepdims=True) + 1e-5)),
    ('rms_norm', lambda t: F.rms_norm(t, [6]) if hasattr(F, 'rms_norm') else paddle.incubate.nn.functional.fused_rms_norm(
        t, paddle.ones([6], 'float64'), None, 1e-5, 1)[0], lambda x: x / np.sqrt((x ** 2).mean(-1, keepdims=True) + 1e-5)),
    ('group_norm', lambda t: F.group_norm(t.reshape([2, 6, 1, 2]), 3).reshape([2, 12]) if False else
     F.group_norm(t.reshape([2, 6, 2]), 3).reshape([4, 6]),
     lambda x: ((x.reshape(2, 3, 4) - x.reshape(2, 3, 4).mean(-1, keepdims=True)) /
                np.sqrt(x.reshape(2, 3, 4).var(-1, keepdims=True) + 1e-5)).reshape(4, 6)),
    ('instance_norm', lambda t: F.instance_norm(t.reshape([2, 2, 6])).reshape([4, 6]),
     lambda x: ((x.reshape(2, 2, 6) - x.reshape(2, 2, 6).mean(-1, keepdims=True)) /
                np.sqrt(x.reshape(2, 2, 6).var(-1, keepdims=True) + 1e-5)).reshape(4, 6)),
    ('batch_norm_train', lambda t: F.batch_norm(t, paddle.zeros([6], 'float64'), paddle.ones([6], 'float64'),
                                                training=True),
     lambda x: (x - x.mean(0)) / np.sqrt(x.var(0) + 1e-5)),
]


@pytest.mark.parametrize("name,fn,ref", NORMS, ids=[n[0] for n in NORMS])
def test_norms(name, fn, ref):
    x = _any(4, 6)
    np.testing.assert_allclose(fn(_t(x)).numpy(), ref(x), rtol=1e-5, atol=1e-7)
    _fd_check(fn, [x], rtol=1e-3)


def test_embedding_one_hot_interpolate():
    w = _any(10, 4)
    ids = np.array([[1, 3], [9, 0]])
    np.testing.assert_allclose(F.embedding(_t(ids), _t(w)).numpy(), w[ids])
    _fd_check(lambda t: F.embedding(_t(ids), t), [w])
    np.testing.assert_array_equal(F.one_hot(_t(np.array([0, 2])), 3).numpy(), np.eye(3)[[0, 2]])
    x = _any(1, 1, 2, 2)
    up = F.interpolate(_t(x), scale_factor=2, mode='nearest').numpy()
    np.testing.assert_allclose(up, x.repeat(2, 2).repeat(2, 3))
    _fd_check(lambda t: F.interpolate(t, size=[3, 3], mode='bilinear', align_corners=True), [x])


def test_attention_math():
    q, k, v = _any(1, 4, 2, 8), _any(1, 4, 2, 8), _any(1, 4, 2, 8)
    out = F.scaled_dot_product_attention(_t(q), _t(k), _t(v), is_causal=True).numpy()
    qt, kt, vt = (a.transpose(0, 2, 1, 3) for a in (q, k, v))
    s = qt @ kt.transpose(0, 1, 3, 2) / math.sqrt(8)
    s = s + np.triu(np.full((4, 4), -np.inf), 1)
    ref = (sps.softmax(s, -1) @ vt).transpose(0, 2, 1, 3)
    np.testing.assert_allclose(out, ref, rtol=1e-6, atol=1e-9)
    _fd_check(lambda a, b, c: F.scaled_dot_product_attention(a, b, c, is_causal=True), [q, k, v])


# ----------------------------------------------------------------------------- search / sort / logic
def test_search_sort():
    x = _any(4, 6)
    np.testing.assert_array_equal(paddle.argmax(_t(x), 1).numpy(), x.argmax(1))
    np.testing.assert_array_equal(paddle.argmin(_t(x), 0).numpy(), x.argmin(0))
    np.testing.assert_allclose(paddle.sort(_t(x), 1).numpy(), np.sort(x, 1))
    np.testing.assert_allclose(paddle.sort(_t(x), 1, descending=True).numpy(), -np.sort(-x, 1))
    np.testing.assert_array_equal(paddle.argsort(_t(x), 0).numpy(), np.argsort(x, 0, kind='stable'))
    v, i = paddle.topk(_t(x), 2, axis=1)
    np.testing.assert_allclose(v.numpy(), -np.sort(-x, 1)[:, :2])
    np.testing.assert_allclose(paddle.kthvalue(_t(x), 2, axis=1)[0].numpy(), np.sort(x, 1)[:, 1])
    np.testing.assert_allclose(paddle.median(_t(x), axis=1).numpy(), np.median(x, 1))
    np.testing.assert_allclose(paddle.quantile(_t(x), 0.3, axis=1).numpy(), np.quantile(x, 0.3, 1), rtol=1e-6)
    np.testing.assert_array_equal(paddle.searchsorted(_t(np.sort(x[0])), _t(x[1])).numpy(),
                                  np.searchsorted(np.sort(x[0]), x[1]))
    np.testing.assert_array_equal(paddle.nonzero(_t(x > 0)).numpy(), np.argwhere(x > 0))
    np.testing.assert_array_equal(paddle.masked_select(_t(x), _t(x > 0)).numpy(), x[x > 0])
    u = paddle.unique(_t(np.array([3, 1, 3, 2, 1])))
    np.testing.assert_array_equal(u.numpy(), [1, 2, 3])
    np.testing.assert_array_equal(paddle.bincount(_t(np.array([0, 1, 1, 3]))).numpy(), [1, 2, 0, 1])
    np.testing.assert_allclose(paddle.histogram(_t(x), bins=4, min=-2, max=2).numpy(),
                               np.histogram(x, 4, (-2, 2))[0])
    np.testing.assert_array_equal(paddle.mode(_t(np.array([[1, 2, 2, 3]])), axis=1)[0].numpy(), [2])


COMPARE = [('equal', np.equal), ('not_equal', np.not_equal), ('less_than', np.less), ('less_equal', np.less_equal),
           ('greater_than', np.greater), ('greater_equal', np.greater_equal)]


@pytest.mark.parametrize("name,ref", COMPARE, ids=[c[0] for c in COMPARE])
def test_compare(name, ref):
    a = np.round(_any(3, 4))
    b = np.round(_any(3, 4))
    np.testing.assert_array_equal(getattr(paddle, name)(_t(a), _t(b)).numpy(), ref(a, b))


LOGIC = [('logical_and', np.logical_and), ('logical_or', np.logical_or), ('logical_xor', np.logical_xor),
         ('bitwise_and', np.bitwise_and), ('bitwise_or', np.bitwise_or), ('bitwise_xor', np.bitwise_xor)]


@pytest.mark.parametrize("name,ref", LOGIC, ids=[c[0] for c in LOGIC])
def test_logic(name, ref):
    if name.startswith('bitwise'):
        a, b = R.randint(0, 16, (3, 4)), R.randint(0, 16, (3, 4))
    else:
        a, b = R.rand(3, 4) > 0.5, R.rand(3, 4) > 0.5
    np.testing.assert_array_equal(getattr(paddle, name)(_t(a), _t(b)).numpy(), ref(a, b))


def test_isclose_allclose_equal_all():
    a = _any(3, 3)
    assert bool(paddle.allclose(_t(a), _t(a + 1e-10)))
    assert bool(paddle.equal_all(_t(a), _t(a)))
    np.testing.assert_array_equal(paddle.isclose(_t(a), _t(a + 1e-3)).numpy(), np.isclose(a, a + 1e-3))
    np.testing.assert_array_equal(paddle.isnan(_t(np.array([1.0, np.nan]))).numpy(), [False, True])
    np.testing.assert_array_equal(paddle.isinf(_t(np.array([1.0, np.inf]))).numpy(), [False, True])
    np.testing.assert_array_equal(paddle.isfinite(_t(np.array([np.inf, 1.0]))).numpy(), [False, True])


# ----------------------------------------------------------------------------- creation
CREATE = [
    ('zeros', lambda: paddle.zeros([2, 3]), np.zeros((2, 3))),
    ('ones', lambda: paddle.ones([2, 3], 'int32'), np.ones((2, 3), 'int32')),
    ('full', lambda: paddle.full([2, 2], 7.5), np.full((2, 2), 7.5)),
    ('arange', lambda: paddle.arange(1, 10, 3), np.arange(1, 10, 3)),
    ('linspace', lambda: paddle.linspace(0, 1, 5), np.linspace(0, 1, 5)),
    ('logspace', lambda: paddle.logspace(0, 2, 3), np.logspace(0, 2, 3)),
    ('eye', lambda: paddle.eye(3, 4), np.eye(3, 4)),
    ('diag', lambda: paddle.diag(paddle.to_tensor([1.0, 2.0])), np.diag([1.0, 2.0])),
    ('diag_offset', lambda: paddle.diag(paddle.to_tensor([1.0, 2.0]), 1), np.diag([1.0, 2.0], 1)),
    ('diagflat', lambda: paddle.diagflat(paddle.to_tensor([[1.0, 2.0]])), np.diagflat([1.0, 2.0])),
    ('tril_indices', lambda: paddle.tril_indices(3, 3), np.stack(np.tril_indices(3))),
    ('triu_indices', lambda: paddle.triu_indices(3, 3, 1), np.stack(np.triu_indices(3, 1))),
    ('meshgrid', lambda: paddle.meshgrid(paddle.arange(2), paddle.arange(3))[0], np.meshgrid(np.arange(2),
                                                                                             np.arange(3),
                                                                                             indexing='ij')[0]),
    ('full_like', lambda: paddle.full_like(paddle.ones([2]), 3), np.full(2, 3.0)),
    ('zeros_like', lambda: paddle.zeros_like(paddle.ones([2, 1])), np.zeros((2, 1))),
    ('empty_shape', lambda: paddle.to_tensor(list(paddle.empty([3, 2]).shape)), np.array([3, 2])),
    ('complex', lambda: paddle.abs(paddle.complex(paddle.to_tensor([3.0]), paddle.to_tensor([4.0]))), np.array([5.0])),
    ('polar', lambda: paddle.real(paddle.polar(paddle.to_tensor([2.0]), paddle.to_tensor([0.0]))), np.array([2.0])),
    ('vander', lambda: paddle.vander(paddle.to_tensor([1.0, 2.0, 3.0])), np.vander([1.0, 2.0, 3.0])),
]


@pytest.mark.parametrize("name,fn,ref", CREATE, ids=[c[0] for c in CREATE])
def test_creation(name, fn, ref):
    out = fn()
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-6)


def test_random_distributions_shapes_and_moments():
    paddle.seed(0)
    u = paddle.uniform([20000], min=-1, max=3).numpy()
    assert abs(u.mean() - 1) < 0.05 and u.min() >= -1 and u.max() <= 3
    n = paddle.normal(1.0, 2.0, [20000]).numpy()
    assert abs(n.mean() - 1) < 0.1 and abs(n.std() - 2) < 0.1
    assert paddle.randint(0, 5, [100]).numpy().max() < 5
    p = paddle.randperm(10).numpy()
    assert sorted(p.tolist()) == list(range(10))
    b = paddle.bernoulli(paddle.full([20000], 0.3)).numpy()
    assert abs(b.mean() - 0.3) < 0.02
    m = paddle.multinomial(paddle.to_tensor([0.0, 1.0, 0.0]), 5, replacement=True).numpy()
    assert (m == 1).all()
    po = paddle.poisson(paddle.full([20000], 4.0)).numpy()
    assert abs(po.mean() - 4) < 0.1


# ----------------------------------------------------------------------------- dtype / cast semantics
@pytest.mark.parametrize("src,dst", [('float32', 'float64'), ('float64', 'float32'), ('float32', 'int32'),
                                     ('int64', 'float32'), ('float32', 'bfloat16'), ('float32', 'float16'),
                                     ('bool', 'float32'), ('int32', 'bool')])
def test_cast(src, dst):
    x = (_any(3, 4) * 3)
    if src == 'bool':
        x = x > 0
    t = paddle.to_tensor(x.astype(src) if src != 'bfloat16' else x).astype(dst)
    assert str(t.dtype).split('.')[-1] == dst
    ref = x.astype(src).astype('float32' if dst in ('bfloat16', 'float16') else dst)
    tol = 1e-2 if dst in ('bfloat16', 'float16') else 0
    np.testing.assert_allclose(t.astype('float32').numpy() if dst in ('bfloat16', 'float16') else t.numpy(),
                               ref, rtol=tol, atol=tol)


@pytest.mark.parametrize("a_dt,b_dt,res", [('float32', 'float64', 'float64'), ('int32', 'float32', 'float32'),
                                           ('int64', 'int32', 'int64'), ('float16', 'float32', 'float32'),
                                           ('bool', 'int32', 'int32')])
def test_type_promotion(a_dt, b_dt, res):
    a = paddle.ones([2], a_dt)
    b = paddle.ones([2], b_dt)
    assert str((a + b).dtype).split('.')[-1] == res


# ----------------------------------------------------------------------------- autograd semantics
def test_grad_accumulates_and_stop_gradient():
    x = _t(_any(3), True)
    y = (x * x).sum()
    y.backward()
    g1 = x.grad.numpy().copy()
    (x * 3).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), g1 + 3)
    z = _t(_any(3))
    assert z.stop_gradient
    w = x.detach()
    assert w.stop_gradient


def test_higher_order_grad():
    x = _t(np.array([1.5, -0.5]), True)
    y = (x ** 3).sum()
    g, = paddle.grad([y], [x], create_graph=True)
    g2, = paddle.grad([g.sum()], [x])
    np.testing.assert_allclose(g2.numpy(), 6 * np.array([1.5, -0.5]))


def test_pylayer_custom_backward():
    class Cube(paddle.autograd.PyLayer):
        @staticmethod
        def forward(ctx, x):
            ctx.save_for_backward(x)
            return x ** 3

        @staticmethod
        def backward(ctx, dy):
            x, = ctx.saved_tensor()
            return dy * 3 * x ** 2
    x = _any(4)
    _fd_check(lambda t: Cube.apply(t), [x])
