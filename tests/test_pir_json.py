"""The reference's PIR program format (<prefix>.json, static/pir_json.py; reference
python/paddle/static/pir_io.py:527 save_pir / :610 load_pir, schema
paddle/fluid/pir/serialize_deserialize/include/schema.h):

* round trips: a CNN and an embedding / transformer-style net saved as PIR JSON (format='pir',
  FLAGS_enable_pir_api for jit.save) load back through load_inference_model, jit.load and
  paddle.inference and reproduce the recorded program's outputs;
* spec-built fixtures: for every operation of the importable set, a program written by hand from the
  schema (pd_op.data -> op -> pd_op.fetch, mutable attributes as pd_op.full / full_int_array
  operands, vectors through builtin.combine / builtin.split) runs and matches numpy.
Parity with files written by the reference itself is unpinned (no reference build here)."""
import json

import numpy as np
import pytest
import scipy.special as sps
import torch

import paddle
import paddle.static as static
import paddle.nn.functional as F
from paddle.static import proto as P, pir_json


def _ops(path):
    doc = json.load(open(path))
    assert doc['base_code']['magic'] == 'pir'
    return [op['#'] for op in doc['program']['regions'][0]['blocks'][0]['ops']], doc


def test_cnn_pir_round_trip(static_mode, tmp_path):
    paddle.seed(0)
    main = static.Program()
    with static.program_guard(main):
        x = static.data('img', [None, 3, 8, 8], 'float32')
        c = static.nn.conv2d(x, 4, 3, padding=1, act='relu')
        p = F.max_pool2d(c, 2, 2)
        b = static.nn.batch_norm(p, is_test=True)
        a = F.adaptive_avg_pool2d(b, 1)
        f = paddle.flatten(a, 1)
        out = static.nn.fc(f, 5)
        prob = F.softmax(F.gelu(F.layer_norm(out, [5])) * 2.0 + 1.0)
    exe = static.Executor(paddle.CPUPlace())
    xs = np.random.rand(2, 3, 8, 8).astype('float32')
    ref, = exe.run(main, feed={'img': xs}, fetch_list=[prob])
    prefix = str(tmp_path / 'cnn')
    static.save_inference_model(prefix, [x], [prob], exe, program=main, format='pir')
    ops, doc = _ops(prefix + '.json')
    for t in ('p', '1.data', '1.conv2d', '1.relu', '1.pool2d', '1.full_int_array', '1.batch_norm', '1.flatten',
              '1.matmul', '1.add', '1.layer_norm', '1.gelu', '1.scale', '1.full', '1.softmax', '1.fetch'):
        assert t in ops, (t, ops)
    data = [o for o in doc['program']['regions'][0]['blocks'][0]['ops'] if o['#'] == '1.data'][0]
    assert data['O'][0]['TT']['D'][1] == [-1, 3, 8, 8]
    prog, feeds, fetches = static.load_inference_model(prefix, exe)
    assert feeds == ['img']
    got, = exe.run(prog, feed={'img': xs}, fetch_list=fetches)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
    got3, = exe.run(prog, feed={'img': np.concatenate([xs, xs, xs])}, fetch_list=fetches)
    assert got3.shape == (6, 5)


def test_jit_save_pir_flag_and_predictor(tmp_path):
    class Net(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.emb = paddle.nn.Embedding(20, 8)
            self.fc1 = paddle.nn.Linear(8, 16)
            self.fc2 = paddle.nn.Linear(16, 4)

        def forward(self, ids):
            h = self.emb(ids).mean(1)
            h = paddle.tanh(self.fc1(h))
            return F.softmax(self.fc2(h).reshape([-1, 2, 2]).transpose([0, 2, 1]), -1)
    net = Net()
    net.eval()
    path = str(tmp_path / 'net')
    paddle.set_flags({'FLAGS_enable_pir_api': True})
    try:
        paddle.jit.save(net, path, input_spec=[static.InputSpec([None, 5], 'int64', 'ids')])
    finally:
        paddle.set_flags({'FLAGS_enable_pir_api': False})
    ops, _ = _ops(path + '.json')
    assert '1.embedding' in ops and '1.mean' in ops and '1.transpose' in ops and '1.reshape' in ops
    ids = np.random.randint(0, 20, (3, 5)).astype('int64')
    ref = net(paddle.to_tensor(ids)).numpy()
    from paddle import inference
    pred = inference.create_predictor(inference.Config(path + '.json', path + '.pdiparams'))
    h = pred.get_input_handle(pred.get_input_names()[0])
    h.copy_from_cpu(ids)
    pred.run()
    out = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)
    loaded = paddle.jit.load(path)
    np.testing.assert_allclose(loaded(paddle.to_tensor(ids)).numpy(), ref, rtol=1e-5, atol=1e-6)


# ----------------------------------------------------------------------------- spec fixtures
class _B:
    """Writes a PIR JSON program straight from the schema (independent of the exporter)."""

    def __init__(self):
        self.ops, self.nid, self.params = [], 1, []

    @staticmethod
    def tt(dt, shape):
        return {'#': '0.t_dtensor', 'D': [{'#': '0.t_' + dt}, list(shape), 'NCHW', [], 0]}

    def _new(self):
        v = self.nid
        self.nid += 1
        return v

    def op(self, name, ins, attrs=(), nout=1, tts=None):
        outs = [self._new() for _ in range(nout)]
        tts = tts or [self.tt('f32', [])] * nout
        self.ops.append({'#': name, 'I': [{'%': i} for i in ins], 'O': [{'%': o, 'TT': t} for o, t in zip(outs, tts)],
                         'A': [{'N': k, 'AT': v} for k, v in attrs]})
        return outs if nout != 1 else outs[0]

    def param(self, name, arr):
        v = self._new()
        self.ops.append({'#': 'p', 'O': {'%': v, 'TT': self.tt('f32', arr.shape)}, 'A': [0, 1, 1, name]})
        self.params.append((name, arr))
        return v

    def data(self, name, shape, dt='float32'):
        return self.op('1.data', [], [('name', {'#': '0.a_str', 'D': name}),
                                      ('shape', {'#': '1.a_intarray', 'D': list(shape)}),
                                      ('dtype', {'#': '1.a_dtype', 'D': dt}),
                                      ('place', {'#': '1.a_place', 'D': [1, 0, '']})],
                       tts=[self.tt({'float32': 'f32', 'int64': 'i64', 'bool': 'bool'}[dt], shape)])

    def ints(self, vals):
        return self.op('1.full_int_array', [], [('value', {'#': '0.a_array', 'D': [{'#': '0.a_i64', 'D': v}
                                                                                    for v in vals]}),
                                                ('dtype', {'#': '1.a_dtype', 'D': 'int64'}),
                                                ('place', {'#': '1.a_place', 'D': [1, 0, '']})])

    def scalar(self, v, dt='float32'):
        return self.op('1.full', [], [('shape', {'#': '1.a_intarray', 'D': [1]}),
                                      ('value', {'#': '0.a_f64', 'D': float(v)}),
                                      ('dtype', {'#': '1.a_dtype', 'D': dt}),
                                      ('place', {'#': '1.a_place', 'D': [1, 0, '']})])

    def fetch(self, vals):
        for i, v in enumerate(vals):
            self.op('1.fetch', [v], [('name', {'#': '0.a_str', 'D': f'out{i}'}), ('col', {'#': '0.a_i32', 'D': i})])

    def write(self, prefix):
        doc = {'base_code': {'magic': 'pir', 'version': 1, 'trainable': False},
               'program': {'regions': [{'#': 'region_0', 'blocks': [{'#': 'block_0', 'args': [], 'ops': self.ops}]}]}}
        open(prefix + '.json', 'w').write(json.dumps(doc))
        open(prefix + '.pdiparams', 'wb').write(P.save_combine([(n, torch.from_numpy(a)) for n, a in
                                                                sorted(self.params)]))


def _bool(v):
    return {'#': '0.a_bool', 'D': v}


def _i32(v):
    return {'#': '0.a_i32', 'D': v}


def _f32(v):
    return {'#': '0.a_f32', 'D': v}


def _str(v):
    return {'#': '0.a_str', 'D': v}


def _arr(vals, k='0.a_i32'):
    return {'#': '0.a_array', 'D': [{'#': k, 'D': v} for v in vals]}


R = np.random.RandomState(0)
X = R.rand(2, 3, 4).astype('float32') + 0.1
Y = R.rand(2, 3, 4).astype('float32') + 0.1
IMG = R.rand(2, 3, 6, 6).astype('float32')

# (op, builder(b, x, y) -> outputs, numpy reference(x, y) -> outputs, inputs)
CASES = {
    'relu': (lambda b, x, y: b.op('1.relu', [x]), lambda x, y: np.maximum(x, 0)),
    'tanh': (lambda b, x, y: b.op('1.tanh', [x]), lambda x, y: np.tanh(x)),
    'sigmoid': (lambda b, x, y: b.op('1.sigmoid', [x]), lambda x, y: sps.expit(x)),
    'exp': (lambda b, x, y: b.op('1.exp', [x]), lambda x, y: np.exp(x)),
    'sqrt': (lambda b, x, y: b.op('1.sqrt', [x]), lambda x, y: np.sqrt(x)),
    'log': (lambda b, x, y: b.op('1.log', [x]), lambda x, y: np.log(x)),
    'square': (lambda b, x, y: b.op('1.square', [x]), lambda x, y: x * x),
    'sin': (lambda b, x, y: b.op('1.sin', [x]), lambda x, y: np.sin(x)),
    'silu': (lambda b, x, y: b.op('1.silu', [x]), lambda x, y: x * sps.expit(x)),
    'gelu': (lambda b, x, y: b.op('1.gelu', [x], [('approximate', _bool(False))]),
             lambda x, y: 0.5 * x * (1 + sps.erf(x / np.sqrt(2)))),
    'softmax': (lambda b, x, y: b.op('1.softmax', [x], [('axis', _i32(-1))]), lambda x, y: sps.softmax(x, -1)),
    'leaky_relu': (lambda b, x, y: b.op('1.leaky_relu', [x], [('negative_slope', _f32(0.1))]),
                   lambda x, y: np.where(x > 0, x, 0.1 * x)),
    'add': (lambda b, x, y: b.op('1.add', [x, y]), lambda x, y: x + y),
    'subtract': (lambda b, x, y: b.op('1.subtract', [x, y]), lambda x, y: x - y),
    'multiply': (lambda b, x, y: b.op('1.multiply', [x, y]), lambda x, y: x * y),
    'divide': (lambda b, x, y: b.op('1.divide', [x, y]), lambda x, y: x / y),
    'maximum': (lambda b, x, y: b.op('1.maximum', [x, y]), lambda x, y: np.maximum(x, y)),
    'matmul': (lambda b, x, y: b.op('1.matmul', [x, y], [('transpose_x', _bool(False)), ('transpose_y', _bool(True))]),
               lambda x, y: x @ np.swapaxes(y, -1, -2)),
    'scale': (lambda b, x, y: b.op('1.scale', [x, b.scalar(3.0)], [('bias', _f32(0.5)), ('bias_after_scale', _bool(True))]),
              lambda x, y: 3 * x + 0.5),
    'reshape': (lambda b, x, y: b.op('1.reshape', [x, b.ints([0, 12])], nout=2)[0], lambda x, y: x.reshape(2, 12)),
    'transpose': (lambda b, x, y: b.op('1.transpose', [x], [('perm', _arr([2, 0, 1]))]),
                  lambda x, y: x.transpose(2, 0, 1)),
    'concat': (lambda b, x, y: b.op('1.concat', [b.op('0.combine', [x, y]), b.scalar(1, 'int32')]),
               lambda x, y: np.concatenate([x, y], 1)),
    'stack': (lambda b, x, y: b.op('1.stack', [b.op('0.combine', [x, y])], [('axis', _i32(0))]),
              lambda x, y: np.stack([x, y], 0)),
    'unsqueeze': (lambda b, x, y: b.op('1.unsqueeze', [x, b.ints([1])], nout=2)[0], lambda x, y: x[:, None]),
    'mean': (lambda b, x, y: b.op('1.mean', [x], [('axis', {'#': '1.a_intarray', 'D': [1]}), ('keepdim', _bool(False))]),
             lambda x, y: x.mean(1)),
    'sum': (lambda b, x, y: b.op('1.sum', [x, b.ints([0, 2])], [('keepdim', _bool(True))]),
            lambda x, y: x.sum((0, 2), keepdims=True)),
    'max': (lambda b, x, y: b.op('1.max', [x, b.ints([-1])], [('keepdim', _bool(False))]), lambda x, y: x.max(-1)),
    'cast': (lambda b, x, y: b.op('1.cast', [x], [('dtype', {'#': '1.a_dtype', 'D': 'int32'})]),
             lambda x, y: (x * 0 + 3.7).astype('int32') * 0 + x.astype('int32')),
    'clip': (lambda b, x, y: b.op('1.clip', [x, b.scalar(0.3), b.scalar(0.6)]), lambda x, y: np.clip(x, 0.3, 0.6)),
    'slice': (lambda b, x, y: b.op('1.slice', [x, b.ints([1]), b.ints([3])],
                                   [('axes', _arr([2], '0.a_i64')), ('infer_flags', _arr([1], '0.a_i64')),
                                    ('decrease_axis', _arr([], '0.a_i64'))]), lambda x, y: x[:, :, 1:3]),
    'flatten': (lambda b, x, y: b.op('1.flatten', [x], [('start_axis', _i32(1)), ('stop_axis', _i32(2))], nout=2)[0],
                lambda x, y: x.reshape(2, 12)),
    'where': (lambda b, x, y: b.op('1.where', [b.op('1.greater_than', [x, y]), x, y]),
              lambda x, y: np.where(x > y, x, y)),
    'tril': (lambda b, x, y: b.op('1.tril', [x], [('diagonal', _i32(0))]), lambda x, y: np.tril(x)),
    'cumsum': (lambda b, x, y: b.op('1.cumsum', [x, b.scalar(2, 'int32')],
                                    [('flatten', _bool(False)), ('exclusive', _bool(False)), ('reverse', _bool(False))]),
               lambda x, y: np.cumsum(x, 2)),
    'expand': (lambda b, x, y: b.op('1.expand', [b.op('1.mean', [x], [('axis', {'#': '1.a_intarray', 'D': [0]}),
                                                                       ('keepdim', _bool(True))]), b.ints([2, 3, 4])]),
               lambda x, y: np.broadcast_to(x.mean(0, keepdims=True), (2, 3, 4))),
    'tile': (lambda b, x, y: b.op('1.tile', [x, b.ints([1, 2, 1])]), lambda x, y: np.tile(x, (1, 2, 1))),
    'topk': (lambda b, x, y: b.op('1.topk', [x, b.scalar(2, 'int32')], [('axis', _i32(-1)), ('largest', _bool(True)),
                                                                       ('sorted', _bool(True))], nout=2)[0],
             lambda x, y: -np.sort(-x, -1)[..., :2]),
    'split': (lambda b, x, y: list(b.op('0.split', [b.op('1.split', [x, b.ints([1, 3]), b.scalar(2, 'int32')])],
                                        nout=2)), lambda x, y: [x[..., :1], x[..., 1:]]),
    'p_norm': (lambda b, x, y: b.op('1.p_norm', [x], [('porder', _f32(2.0)), ('axis', _i32(-1)), ('epsilon', _f32(1e-12)),
                                                      ('keepdim', _bool(False)), ('asvector', _bool(False))]),
               lambda x, y: np.linalg.norm(x, axis=-1)),
}


@pytest.mark.parametrize('name', sorted(CASES))
def test_spec_built_pir_op(name, tmp_path):
    build, ref = CASES[name]
    b = _B()
    x = b.data('x', [-1, 3, 4])
    y = b.data('y', [-1, 3, 4])
    outs = build(b, x, y)
    outs = outs if isinstance(outs, list) else [outs]
    b.fetch(outs)
    prefix = str(tmp_path / name)
    b.write(prefix)
    exe = static.Executor(paddle.CPUPlace())
    prog, feeds, fetches = static.load_inference_model(prefix, exe)
    got = exe.run(prog, feed={'x': X, 'y': Y}, fetch_list=fetches)
    want = ref(X, Y)
    want = want if isinstance(want, list) else [want]
    assert len(got) == len(want)
    for g, w in zip(got, want):
        np.testing.assert_allclose(np.asarray(g, dtype=np.float64), np.asarray(w, dtype=np.float64), rtol=1e-5,
                                   atol=1e-6, err_msg=name)


def test_spec_built_pir_cnn_with_parameters(tmp_path):
    """conv2d + batch_norm + pool2d + embedding-free head from the schema, parameters as
    builtin.parameter ops filled from the .pdiparams stream."""
    rng = np.random.RandomState(1)
    w = rng.randn(4, 3, 3, 3).astype('float32') * 0.3
    mean, var = rng.rand(4).astype('float32'), rng.rand(4).astype('float32') + 0.5
    sc, bi = rng.rand(4).astype('float32'), rng.rand(4).astype('float32')
    fw = rng.randn(4, 2).astype('float32')
    b = _B()
    pw, pm, pv, ps, pb, pf = (b.param(n, a) for n, a in (('conv.w', w), ('bn.mean', mean), ('bn.var', var),
                                                         ('bn.scale', sc), ('bn.bias', bi), ('fc.w', fw)))
    x = b.data('img', [-1, 3, 6, 6])
    c = b.op('1.conv2d', [x, pw], [('strides', _arr([1, 1])), ('paddings', _arr([1, 1])),
                                   ('padding_algorithm', _str('EXPLICIT')), ('dilations', _arr([1, 1])),
                                   ('groups', _i32(1)), ('data_format', _str('NCHW'))])
    bn = b.op('1.batch_norm', [c, pm, pv, ps, pb], [('is_test', _bool(True)), ('momentum', _f32(0.9)),
                                                    ('epsilon', _f32(1e-5)), ('data_format', _str('NCHW')),
                                                    ('use_global_stats', _bool(True)),
                                                    ('trainable_statistics', _bool(False))], nout=6)[0]
    r = b.op('1.relu', [bn])
    pl = b.op('1.pool2d', [r, b.ints([1, 1])], [('strides', _arr([1, 1])), ('paddings', _arr([0, 0])),
                                                 ('ceil_mode', _bool(False)), ('exclusive', _bool(True)),
                                                 ('data_format', _str('NCHW')), ('pooling_type', _str('avg')),
                                                 ('global_pooling', _bool(False)), ('adaptive', _bool(True)),
                                                 ('padding_algorithm', _str('EXPLICIT'))])
    f = b.op('1.flatten', [pl], [('start_axis', _i32(1)), ('stop_axis', _i32(3))], nout=2)[0]
    o = b.op('1.matmul', [f, pf], [('transpose_x', _bool(False)), ('transpose_y', _bool(False))])
    b.fetch([o])
    prefix = str(tmp_path / 'cnn')
    b.write(prefix)
    from paddle import inference
    pred = inference.create_predictor(inference.Config(prefix + '.json', prefix + '.pdiparams'))
    out = pred.run([paddle.to_tensor(IMG)])[0].numpy()
    t = torch.nn.functional.conv2d(torch.from_numpy(IMG), torch.from_numpy(w), padding=1)
    t = (t - torch.from_numpy(mean)[:, None, None]) / torch.sqrt(torch.from_numpy(var)[:, None, None] + 1e-5)
    t = torch.relu(t * torch.from_numpy(sc)[:, None, None] + torch.from_numpy(bi)[:, None, None])
    ref = t.mean((2, 3)).numpy() @ fw
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-5)


def test_not_pir_json_rejected():
    with pytest.raises(ValueError):
        pir_json.load(b'{"base_code": {"magic": "other"}, "program": {}}')
