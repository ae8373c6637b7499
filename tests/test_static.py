"""Static graph: Program recording, Executor training, control flow, inference-model IO."""
import numpy as np
import pytest

import paddle
import paddle.static as static


def test_static_mlp_trains_and_matches_dygraph(static_mode):
    paddle.seed(7)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 8], 'float32')
        y = static.data('y', [None, 1], 'int64')
        assert x.shape == [-1, 8]
        h = static.nn.fc(x, 16, activation='relu')
        logits = static.nn.fc(h, 3)
        loss = paddle.nn.functional.cross_entropy(logits, y.squeeze(-1)).mean() if False else \
            paddle.nn.functional.cross_entropy(logits, y)
        opt = paddle.optimizer.SGD(learning_rate=0.5)
        opt.minimize(loss)
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    rng = np.random.RandomState(0)
    xs = rng.randn(64, 8).astype('float32')
    ys = (xs[:, :3].argmax(1)).reshape(-1, 1).astype('int64')
    losses = []
    for i in range(30):
        lv, = exe.run(main, feed={'x': xs, 'y': ys}, fetch_list=[loss])
        losses.append(float(lv))
    assert losses[-1] < losses[0] * 0.7, losses
    # a different batch size runs through the same program (sentinel re-specialisation)
    out, = exe.run(main.clone(for_test=True), feed={'x': xs[:5], 'y': ys[:5]}, fetch_list=[logits])
    assert out.shape == (5, 3)


def test_static_reshape_with_dynamic_dims(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, None, 4], 'float32')
        b, s = x.shape[0], x.shape[1]
        assert (b, s) == (-1, -1)
        y = x.reshape([-1, 4]) * 2.0
        z = paddle.matmul(y, paddle.ones([4, 2]))
        n = paddle.arange(0, 10)[:3]
    exe = static.Executor(paddle.CPUPlace())
    a = np.random.rand(3, 5, 4).astype('float32')
    zv, nv = exe.run(main, feed={'x': a}, fetch_list=[z, n])
    np.testing.assert_allclose(zv, (a.reshape(-1, 4) * 2) @ np.ones((4, 2)), rtol=1e-5)
    assert nv.tolist() == [0, 1, 2]


def test_static_constants_are_not_taken_for_dynamic_dims(static_mode):
    """Integers in a program that share a factor with small dynamic-dim sentinels (19946 = 2 * 9973,
    the round-1 batch sentinel) must run unchanged at any feed shape."""
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, 4], 'float32')
        n = paddle.arange(0, 19946).sum()
        y = x.sum() + paddle.ones([9967 * 2, 1]).sum()
    exe = static.Executor(paddle.CPUPlace())
    a = np.ones((3, 4), 'float32')
    nv, yv = exe.run(main, feed={'x': a}, fetch_list=[n, y])
    assert int(nv) == 19946 * 19945 // 2
    assert float(yv) == 12.0 + 9967 * 2


def test_static_cond_and_while(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [1], 'float32')
        out = static.nn.cond(x.sum() > 0, lambda: x * 10, lambda: x - 10)
        i = paddle.zeros([1], 'int64')
        ten = paddle.full([1], 5, 'int64')
        i_out, acc = static.nn.while_loop(lambda i, a: i < ten, lambda i, a: [i + 1, a + x], [i, x * 0])
    exe = static.Executor(paddle.CPUPlace())
    o1, a1 = exe.run(main, feed={'x': np.array([2.0], 'float32')}, fetch_list=[out, acc])
    o2, = exe.run(main, feed={'x': np.array([-1.0], 'float32')}, fetch_list=[out])
    assert o1.tolist() == [20.0] and o2.tolist() == [-11.0] and a1.tolist() == [10.0]


def test_gradients_and_append_backward(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [3], 'float32')
        x.stop_gradient = False
        w = static.create_parameter([3], 'float32')
        y = (x * x * w).sum()
        gx, = static.gradients(y, [x])
        pg = static.append_backward(y, parameter_list=[w])
    exe = static.Executor(paddle.CPUPlace())
    xv = np.array([1.0, 2.0, 3.0], 'float32')
    g, gw = exe.run(main, feed={'x': xv}, fetch_list=[gx, pg[0][1]])
    np.testing.assert_allclose(g, 2 * xv * w.numpy(), rtol=1e-5)
    np.testing.assert_allclose(gw, xv * xv, rtol=1e-5)


def test_save_load_inference_model(static_mode, tmp_path):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('img', [None, 1, 8, 8], 'float32')
        c = static.nn.conv2d(x, 4, 3, padding=1, act='relu')
        f = paddle.flatten(c, 1)
        out = static.nn.fc(f, 5)
        prob = paddle.nn.functional.softmax(out)
    exe = static.Executor(paddle.CPUPlace())
    a = np.random.rand(2, 1, 8, 8).astype('float32')
    ref, = exe.run(main, feed={'img': a}, fetch_list=[prob])
    prefix = str(tmp_path / 'infer' / 'model')
    static.save_inference_model(prefix, [x], [prob], exe, program=main)
    prog, feeds, fetches = static.load_inference_model(prefix, exe)
    assert feeds == ['img']
    got, = exe.run(prog, feed={'img': a}, fetch_list=fetches)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6)
    got3, = exe.run(prog, feed={'img': np.concatenate([a, a, a])}, fetch_list=fetches)
    assert got3.shape == (6, 5)


class _Net(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc1 = paddle.nn.Linear(6, 12)
        self.ln = paddle.nn.LayerNorm(12)
        self.fc2 = paddle.nn.Linear(12, 3)

    def forward(self, x):
        h = paddle.nn.functional.gelu(self.ln(self.fc1(x)))
        b, d = x.shape[0], h.shape[-1]
        return paddle.nn.functional.softmax(self.fc2(h.reshape([b, d])), -1)


def test_jit_to_static_save_load_roundtrip(tmp_path):
    net = _Net()
    net.eval()
    snet = paddle.jit.to_static(net, input_spec=[static.InputSpec([None, 6], 'float32', 'x')])
    x = paddle.randn([4, 6])
    ref = snet(x)
    prog = snet.forward.concrete_program.main_program
    assert len(prog.nodes) > 3
    path = str(tmp_path / 'net')
    paddle.jit.save(snet, path)
    loaded = paddle.jit.load(path)
    out = loaded(x)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-5, atol=1e-6)
    out7 = loaded(paddle.randn([7, 6]))
    assert out7.shape == [7, 3]
    assert len(loaded.parameters()) == len(net.parameters())


def test_inference_predictor(tmp_path):
    net = _Net()
    net.eval()
    path = str(tmp_path / 'inf')
    paddle.jit.save(net, path, input_spec=[static.InputSpec([None, 6], 'float32', 'x')])
    from paddle import inference
    cfg = inference.Config(path + '.pdmodel', path + '.pdiparams')
    pred = inference.create_predictor(cfg)
    names = pred.get_input_names()
    h = pred.get_input_handle(names[0])
    a = np.random.rand(2, 6).astype('float32')
    h.reshape(a.shape)
    h.copy_from_cpu(a)
    pred.run()
    o = pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu()
    np.testing.assert_allclose(o, net(paddle.to_tensor(a)).numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
def test_gpu_predictor_hip_graph_and_to_static_graph(tmp_path):
    net = _Net()
    net.eval()
    path = str(tmp_path / 'g')
    paddle.jit.save(net, path, input_spec=[static.InputSpec([4, 6], 'float32', 'x')])
    from paddle import inference
    cfg = inference.Config(path + '.pdmodel', path + '.pdiparams')
    cfg.enable_use_gpu(100, 0)
    cfg.enable_hip_graph()
    pred = inference.create_predictor(cfg)
    a = np.random.rand(4, 6).astype('float32')
    outs = []
    for _ in range(3):
        outs.append(pred.run([paddle.to_tensor(a)])[0].numpy())
    ref = net(paddle.to_tensor(a)).numpy()
    for o in outs:
        np.testing.assert_allclose(o, ref, rtol=1e-4, atol=1e-5)
    g = paddle.jit.to_static(net, backend='hip_graph')
    with paddle.no_grad():
        for _ in range(4):
            y = g(paddle.to_tensor(a))
    np.testing.assert_allclose(y.numpy(), ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("level,dtype", [("O1", "bfloat16"), ("O2", "bfloat16"), ("O2", "float16")])
def test_ernie_static_executor_amp(static_mode, level, dtype):
    """BASELINE config 5 on CPU: ERNIE (tiny) built as a static Program, trained by the Executor
    under static.amp (reference: static/amp/decorator.py decorate + amp_init): O2 casts the
    weights (norms kept fp32) with fp32 master weights; float16 uses dynamic loss scaling."""
    import torch
    from paddle.models import ernie_config, ErnieForSequenceClassification
    paddle.seed(3)
    cfg = ernie_config('ernie-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    S, B = 16, 8
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        ids = static.data('ids', [None, S], 'int64')
        lab = static.data('lab', [None], 'int64')
        model = ErnieForSequenceClassification(cfg, num_classes=2)
        logits = model(ids)
        loss = paddle.nn.functional.cross_entropy(logits, lab)
        opt = paddle.optimizer.AdamW(learning_rate=2e-3, parameters=model.parameters())
        opt = static.amp.decorate(opt, level=level, dtype=dtype, init_loss_scaling=1024.0)
        opt.minimize(loss)
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    opt.amp_init(paddle.CPUPlace())
    low = {'bfloat16': torch.bfloat16, 'float16': torch.float16}[dtype]
    dts = {p.name: p._t.dtype for p in main.all_parameters()}
    if level == 'O2':
        assert any(d == low for d in dts.values())
        assert all(d == torch.float32 for n, d in dts.items() if 'norm' in (n or '').lower())
    else:
        assert all(d == torch.float32 for d in dts.values())
    rng = np.random.RandomState(0)
    x = rng.randint(1, cfg.vocab_size, size=(B, S)).astype('int64')
    y = (x[:, 0] % 2).astype('int64')
    losses = []
    for _ in range(25):
        lv, = exe.run(main, feed={'ids': x, 'lab': y}, fetch_list=[loss])
        losses.append(float(lv))
    assert np.isfinite(losses).all(), losses
    assert losses[-1] < losses[0] * 0.6, losses
    if dtype == 'float16':
        assert float(opt.get_loss_scaling()[0]) > 0


@pytest.mark.gpu
def test_ernie_static_executor_amp_o2_gpu(static_mode):
    """BASELINE config 5 on the MI355X: ERNIE static Program + Executor, AMP-O2 bf16."""
    import torch
    from paddle.models import ernie_config, ErnieForSequenceClassification
    paddle.set_device('gpu')
    try:
        paddle.seed(3)
        cfg = ernie_config('ernie-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
        S, B = 64, 16
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            ids = static.data('ids', [None, S], 'int64')
            lab = static.data('lab', [None], 'int64')
            model = ErnieForSequenceClassification(cfg, num_classes=2)
            loss = paddle.nn.functional.cross_entropy(model(ids), lab)
            opt = paddle.optimizer.AdamW(learning_rate=2e-3, parameters=model.parameters())
            opt = static.amp.decorate(opt, level='O2', dtype='bfloat16')
            opt.minimize(loss)
        exe = static.Executor(paddle.CUDAPlace(0))
        exe.run(startup)
        opt.amp_init(paddle.CUDAPlace(0))
        assert any(p._t.dtype == torch.bfloat16 and p._t.is_cuda for p in main.all_parameters())
        rng = np.random.RandomState(0)
        x = rng.randint(1, cfg.vocab_size, size=(B, S)).astype('int64')
        y = (x[:, 0] % 2).astype('int64')
        losses = [float(exe.run(main, feed={'ids': x, 'lab': y}, fetch_list=[loss])[0]) for _ in range(25)]
        assert np.isfinite(losses).all() and losses[-1] < losses[0] * 0.6, losses
    finally:
        paddle.set_device('cpu')


def test_static_auc_and_ctr_metric_bundle():
    """static.auc accumulates ROC histograms across Executor runs (global AUC == the dygraph
    paddle.metric.Auc over all batches; batch AUC over the last slide_steps batches) and
    ctr_metric_bundle accumulates its six sums."""
    import numpy as np
    import paddle
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            pred = paddle.static.data('pred', [None, 2], 'float32')
            lab = paddle.static.data('lab', [None, 1], 'int64')
            auc_out, batch_auc, stats = paddle.static.auc(pred, lab, num_thresholds=255, slide_steps=2)
            sq, ab, pr, q, pos, ins = paddle.static.ctr_metric_bundle(pred[:, 1:2], lab)
        exe = paddle.static.Executor()
        rs = np.random.RandomState(0)
        ref = paddle.metric.Auc(num_thresholds=255)
        ref_last2 = []
        tot = np.zeros(6)
        for _ in range(4):
            y = rs.randint(0, 2, (64, 1)).astype('int64')
            p1 = np.clip(0.5 * y[:, 0] + 0.5 * rs.rand(64), 0, 1).astype('float32')
            pv = np.stack([1 - p1, p1], 1)
            a, b, s_sq, s_pos, s_ins = exe.run(main, feed={'pred': pv, 'lab': y},
                                               fetch_list=[auc_out, batch_auc, sq, pos, ins])
            ref.update(pv, y)
            ref_last2 = (ref_last2 + [(pv, y)])[-2:]
            tot += [((p1 - y[:, 0]) ** 2).sum(), 0, 0, 0, y.sum(), 64]
        np.testing.assert_allclose(float(a), ref.accumulate(), rtol=1e-5)
        r2 = paddle.metric.Auc(num_thresholds=255)
        for pv, y in ref_last2:
            r2.update(pv, y)
        np.testing.assert_allclose(float(b), r2.accumulate(), rtol=1e-5)
        np.testing.assert_allclose(float(s_sq.reshape(-1)[0]), tot[0], rtol=1e-4)
        assert float(s_pos.reshape(-1)[0]) == tot[4] and float(s_ins.reshape(-1)[0]) == tot[5]
    finally:
        paddle.disable_static()
