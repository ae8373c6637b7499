"""Reference program format: ProgramDesc .pdmodel + LoDTensor .pdiparams (static/pdmodel.py,
static/proto.py; reference paddle/fluid/framework/framework.proto:264, static/io.py:470)."""
import numpy as np
import pytest
import scipy.special as sps

import paddle
import paddle.static as static
import paddle.nn.functional as F
from paddle.static import proto as P


def _ops(path):
    d = P.ProgramDesc()
    d.ParseFromString(open(path, 'rb').read())
    return [op.type for op in d.blocks[0].ops], d


def test_cnn_exports_program_desc_and_round_trips(static_mode, tmp_path):
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
    static.save_inference_model(prefix, [x], [prob], exe, program=main)
    ops, desc = _ops(prefix + '.pdmodel')
    assert ops[0] == 'feed' and ops[-1] == 'fetch'
    for t in ('conv2d', 'relu', 'pool2d', 'batch_norm', 'flatten_contiguous_range', 'matmul_v2', 'elementwise_add',
              'layer_norm', 'gelu', 'scale', 'softmax'):
        assert t in ops, (t, ops)
    feed_var = [v for v in desc.blocks[0].vars if v.name == 'img'][0]
    assert list(feed_var.type.lod_tensor.tensor.dims) == [-1, 3, 8, 8]
    # .pdiparams is the LoDTensor stream of the persistables in sorted-name order
    persist = sorted(v.name for v in desc.blocks[0].vars if v.persistable and v.type.type == 7)
    params = P.load_combine(open(prefix + '.pdiparams', 'rb').read(), persist)
    assert len(params) == len(persist) >= 6
    prog, feeds, fetches = static.load_inference_model(prefix, exe)
    assert feeds == ['img']
    got, = exe.run(prog, feed={'img': xs}, fetch_list=fetches)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
    got3, = exe.run(prog, feed={'img': np.concatenate([xs, xs, xs])}, fetch_list=fetches)
    assert got3.shape == (6, 5)


def test_jit_save_is_program_desc_and_predictor_runs(tmp_path):
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
    paddle.jit.save(net, path, input_spec=[static.InputSpec([None, 5], 'int64', 'ids')])
    ops, _ = _ops(path + '.pdmodel')
    assert 'lookup_table_v2' in ops and 'reduce_mean' in ops and 'transpose2' in ops
    ids = np.random.randint(0, 20, (3, 5)).astype('int64')
    ref = net(paddle.to_tensor(ids)).numpy()
    from paddle import inference
    pred = inference.create_predictor(inference.Config(path + '.pdmodel', path + '.pdiparams'))
    h = pred.get_input_handle(pred.get_input_names()[0])
    h.copy_from_cpu(ids)
    pred.run()
    out = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)
    loaded = paddle.jit.load(path)
    np.testing.assert_allclose(loaded(paddle.to_tensor(ids)).numpy(), ref, rtol=1e-5, atol=1e-6)


def _spec_fixture(tmp_path):
    """A model written straight from the format spec (no recorder involved), the way the
    reference's save_inference_model lays it out: feed/fetch ops and vars, mul + elementwise_add
    (axis 1) + relu + matmul_v2 (trans_y) + softmax, persistables in a save_combine stream."""
    rng = np.random.RandomState(3)
    w1, b1, w2 = rng.randn(6, 5).astype('float32'), rng.randn(5).astype('float32'), rng.randn(3, 5).astype('float32')
    d = P.ProgramDesc()
    blk = d.blocks.add()
    blk.idx, blk.parent_idx = 0, -1

    def var(name, typ, dims=None, persist=False, dtype=5):
        v = blk.vars.add()
        v.name, v.persistable = name, persist
        v.type.type = P.VAR_TYPES[typ]
        if typ == 'LOD_TENSOR':
            v.type.lod_tensor.tensor.data_type = dtype
            v.type.lod_tensor.tensor.dims.extend(dims)
    var('feed', 'FEED_MINIBATCH', persist=True)
    var('fetch', 'FETCH_LIST', persist=True)
    var('x', 'LOD_TENSOR', [-1, 6])
    for n, a in (('fc_0.w_0', w1), ('fc_0.b_0', b1), ('fc_1.w_0', w2)):
        var(n, 'LOD_TENSOR', list(a.shape), persist=True)
    for n in ('mul_out', 'add_out', 'relu_out', 'mm_out', 'prob'):
        var(n, 'LOD_TENSOR', [-1, 5])

    def op(typ, ins, outs, **attrs):
        o = blk.ops.add()
        o.type = typ
        for k, vs in ins.items():
            v = o.inputs.add()
            v.parameter = k
            v.arguments.extend(vs)
        for k, vs in outs.items():
            v = o.outputs.add()
            v.parameter = k
            v.arguments.extend(vs)
        for k, val in attrs.items():
            a = o.attrs.add()
            a.name = k
            if isinstance(val, bool):
                a.type, a.b = 6, val
            elif isinstance(val, int):
                a.type, a.i = 0, val
    op('feed', {'X': ['feed']}, {'Out': ['x']}, col=0)
    op('mul', {'X': ['x'], 'Y': ['fc_0.w_0']}, {'Out': ['mul_out']}, x_num_col_dims=1, y_num_col_dims=1)
    op('elementwise_add', {'X': ['mul_out'], 'Y': ['fc_0.b_0']}, {'Out': ['add_out']}, axis=1)
    op('relu', {'X': ['add_out']}, {'Out': ['relu_out']})
    op('matmul_v2', {'X': ['relu_out'], 'Y': ['fc_1.w_0']}, {'Out': ['mm_out']}, trans_x=False, trans_y=True)
    op('softmax', {'X': ['mm_out']}, {'Out': ['prob']}, axis=-1)
    op('fetch', {'X': ['prob']}, {'Out': ['fetch']}, col=0)
    prefix = str(tmp_path / 'spec')
    open(prefix + '.pdmodel', 'wb').write(d.SerializeToString())
    import torch
    open(prefix + '.pdiparams', 'wb').write(P.save_combine([(n, torch.from_numpy(a)) for n, a in
                                                            (('fc_0.w_0', w1), ('fc_0.b_0', b1), ('fc_1.w_0', w2))]))
    return prefix, (w1, b1, w2)


def test_spec_built_program_desc_loads_in_predictor(tmp_path):
    prefix, (w1, b1, w2) = _spec_fixture(tmp_path)
    from paddle import inference
    cfg = inference.Config(prefix + '.pdmodel', prefix + '.pdiparams')
    pred = inference.create_predictor(cfg)
    assert pred.get_input_names() == ['x']
    xs = np.random.rand(4, 6).astype('float32')
    out = pred.run([paddle.to_tensor(xs)])[0].numpy()
    ref = sps.softmax(np.maximum(xs @ w1 + b1, 0) @ w2.T, -1)
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-6)


def test_unsupported_op_falls_back_to_framework_ir(static_mode, tmp_path):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, 4], 'float32')
        y = paddle.cumsum(x, axis=1) * 3.0
    exe = static.Executor(paddle.CPUPlace())
    prefix = str(tmp_path / 'cs')
    static.save_inference_model(prefix, [x], [y], exe, program=main)
    assert open(prefix + '.pdmodel', 'rb').read(1) == b'{'  # this framework's IR
    prog, feeds, fetches = static.load_inference_model(prefix, exe)
    xs = np.random.rand(2, 4).astype('float32')
    np.testing.assert_allclose(exe.run(prog, feed={'x': xs}, fetch_list=fetches)[0], np.cumsum(xs, 1) * 3,
                               rtol=1e-6)


def test_unknown_reference_op_raises(tmp_path):
    d = P.ProgramDesc()
    blk = d.blocks.add()
    blk.idx, blk.parent_idx = 0, -1
    o = blk.ops.add()
    o.type = 'some_custom_op'
    from paddle.static import pdmodel
    with pytest.raises(NotImplementedError):
        pdmodel.load(d.SerializeToString())
