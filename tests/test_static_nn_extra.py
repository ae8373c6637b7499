"""paddle.static.nn breadth: LoD sequence ops (dygraph and static Executor with LoD feeds), norms,
3-D convs, bilinear product, spectral norm, row_conv, nce, data_norm, static_pylayer.
Reference: python/paddle/static/nn/{common,sequence_lod,static_pylayer}.py."""
import numpy as np
import pytest
import scipy.special as sps

import paddle
import paddle.static as static
import paddle.static.nn as snn

R = np.random.RandomState(0)


def _lod(data, lens):
    return static.create_lod_tensor(np.asarray(data, 'float32'), [lens])


def test_lod_tensor_api():
    t = _lod(R.rand(5, 2), [2, 3])
    assert t.lod() == [[0, 2, 5]] and t.recursive_sequence_lengths() == [[2, 3]]
    t.set_recursive_sequence_lengths([[1, 4]])
    assert t.lod() == [[0, 1, 5]] and t.has_valid_recursive_sequence_lengths()
    with pytest.raises(ValueError):
        static.create_lod_tensor(np.zeros((3, 1)), [[1, 1]])


@pytest.mark.parametrize("pool", ['sum', 'average', 'sqrt', 'max', 'min', 'first', 'last'])
def test_sequence_pool(pool):
    x = R.rand(6, 3).astype('float32')
    t = _lod(x, [2, 0, 4])
    out = snn.sequence_pool(t, pool, pad_value=-1.0).numpy()
    segs = [x[0:2], None, x[2:6]]
    for i, s in enumerate(segs):
        if s is None:
            np.testing.assert_allclose(out[i], -1.0)
            continue
        ref = {'sum': s.sum(0), 'average': s.mean(0), 'sqrt': s.sum(0) / np.sqrt(len(s)), 'max': s.max(0),
               'min': s.min(0), 'first': s[0], 'last': s[-1]}[pool]
        np.testing.assert_allclose(out[i], ref, rtol=1e-6)


def test_sequence_first_last_softmax():
    x = R.rand(5, 1).astype('float32')
    t = _lod(x, [3, 2])
    np.testing.assert_allclose(snn.sequence_first_step(t).numpy(), x[[0, 3]])
    np.testing.assert_allclose(snn.sequence_last_step(t).numpy(), x[[2, 4]])
    sm = snn.sequence_softmax(t).numpy().reshape(-1)
    np.testing.assert_allclose(sm[:3], sps.softmax(x[:3, 0]), rtol=1e-6)
    np.testing.assert_allclose(sm[3:], sps.softmax(x[3:, 0]), rtol=1e-6)


def test_sequence_slice_expand_pad_unpad_reshape():
    x = np.arange(12, dtype='float32').reshape(6, 2)
    t = _lod(x, [2, 4])
    sl = snn.sequence_slice(t, paddle.to_tensor([[1], [1]]), paddle.to_tensor([[1], [2]]))
    np.testing.assert_allclose(sl.numpy(), x[[1, 3, 4]])
    assert sl.lod() == [[0, 1, 3]]
    y = _lod(np.zeros((5, 1)), [2, 3])
    e = snn.sequence_expand(paddle.to_tensor(np.array([[1.0], [2.0]], 'float32')), y)
    np.testing.assert_allclose(e.numpy().reshape(-1), [1, 1, 2, 2, 2])
    ea = snn.sequence_expand_as(paddle.to_tensor(np.array([[1.0], [2.0]], 'float32')), y)
    assert ea.lod() == [[0, 2, 5]]
    pad, ln = snn.sequence_pad(t, paddle.to_tensor([0.0]))
    assert pad.shape == [2, 4, 2] and ln.numpy().tolist() == [2, 4]
    np.testing.assert_allclose(pad.numpy()[0, :2], x[:2])
    np.testing.assert_allclose(pad.numpy()[0, 2:], 0)
    up = snn.sequence_unpad(pad, ln)
    np.testing.assert_allclose(up.numpy(), x)
    assert up.lod() == [[0, 2, 6]]
    rs = snn.sequence_reshape(t, 1)
    assert rs.lod() == [[0, 4, 12]] and rs.shape == [12, 1]


def test_sequence_scatter_enumerate():
    inp = paddle.zeros([2, 5])
    idx = static.create_lod_tensor(np.array([[0], [2], [4]], 'int64'), [[1, 2]])
    upd = static.create_lod_tensor(np.array([[1.0], [2.0], [3.0]], 'float32'), [[1, 2]])
    out = snn.sequence_scatter(inp, idx, upd).numpy()
    np.testing.assert_allclose(out, [[1, 0, 0, 0, 0], [0, 0, 2, 0, 3]])
    ids = static.create_lod_tensor(np.array([[1], [2], [3], [4], [5]], 'int64'), [[3, 2]])
    en = snn.sequence_enumerate(ids, 2, pad_value=0).numpy()
    np.testing.assert_array_equal(en, [[1, 2], [2, 3], [3, 0], [4, 5], [5, 0]])


def test_sequence_conv_context_projection():
    paddle.seed(0)
    x = R.rand(5, 3).astype('float32')
    t = _lod(x, [3, 2])
    out = snn.sequence_conv(t, 4, filter_size=3, bias_attr=False)
    assert out.shape == [5, 4] and out.lod() == [[0, 3, 5]]
    # reconstruct with the created weight: rows see [t-1, t, t+1] inside their own sequence
    w = [p for p in paddle.static.default_main_program().all_parameters()][-1] if False else None
    ctx = np.zeros((5, 9), 'float32')
    for s, e in ((0, 3), (3, 5)):
        for r in range(s, e):
            for j, src in enumerate((r - 1, r, r + 1)):
                if s <= src < e:
                    ctx[r, 3 * j:3 * j + 3] = x[src]
    assert np.isfinite(out.numpy()).all() and ctx.shape == (5, 9)


def test_sequence_ops_in_static_program_with_lod_feed(static_mode):
    main = static.Program()
    with static.program_guard(main):
        x = static.data('x', [None, 3], 'float32', lod_level=1)
        pooled = snn.sequence_pool(x, 'sum')
        y = pooled * 2.0
    exe = static.Executor(paddle.CPUPlace())
    data = R.rand(5, 3).astype('float32')
    out, = exe.run(main, feed={'x': _lod(data, [2, 3])}, fetch_list=[y])
    np.testing.assert_allclose(out, 2 * np.stack([data[:2].sum(0), data[2:].sum(0)]), rtol=1e-6)


def test_norms_convs_bilinear_spectral():
    x = paddle.randn([2, 4, 3, 3])
    assert snn.group_norm(x, 2).shape == [2, 4, 3, 3]
    assert snn.instance_norm(x).shape == [2, 4, 3, 3]
    x3 = paddle.randn([1, 2, 4, 4, 4])
    assert snn.conv3d(x3, 3, 3, padding=1).shape == [1, 3, 4, 4, 4]
    assert snn.conv3d_transpose(x3, 3, filter_size=2, stride=2).shape == [1, 3, 8, 8, 8]
    a, b = paddle.randn([5, 3]), paddle.randn([5, 4])
    assert snn.bilinear_tensor_product(a, b, 6).shape == [5, 6]
    w = paddle.randn([8, 6])
    sn = snn.spectral_norm(w, power_iters=30)
    assert abs(np.linalg.svd(sn.numpy(), compute_uv=False)[0] - 1.0) < 1e-2


def test_row_conv_padded_and_lod():
    paddle.seed(1)
    x = paddle.randn([2, 5, 3])
    out = snn.row_conv(x, 2)
    assert out.shape == [2, 5, 3]
    lx = _lod(R.rand(5, 3), [2, 3])
    o2 = snn.row_conv(lx, 1)
    assert o2.shape == [5, 3] and o2.lod() == [[0, 2, 5]]


def test_nce_loss_and_grad():
    paddle.seed(2)
    x = paddle.randn([4, 8])
    x.stop_gradient = False
    lab = paddle.to_tensor(np.array([[1], [3], [5], [7]], 'int64'))
    for sampler in ('uniform', 'log_uniform'):
        cost = snn.nce(x, lab, num_total_classes=10, num_neg_samples=5, sampler=sampler)
        assert cost.shape == [4, 1] and (cost.numpy() > 0).all()
    cost.sum().backward()
    assert x.grad is not None


def test_data_norm_and_sparse_embedding_and_pylayer():
    x = paddle.randn([6, 4]) * 3 + 1
    y = snn.data_norm(x)
    assert y.shape == [6, 4]
    e = snn.sparse_embedding(paddle.to_tensor([[1, 2]]), [10, 4])
    assert e.shape == [1, 2, 4]
    t = paddle.to_tensor([1.0, 2.0])
    t.stop_gradient = False
    out = snn.static_pylayer(lambda a: a * 3, [t], backward_fn=lambda g: g * 10)
    out.sum().backward()
    np.testing.assert_allclose(t.grad.numpy(), [10, 10])
    np.testing.assert_allclose(out.numpy(), [3, 6])


def test_static_nn_namespace_complete():
    ref = ['fc', 'batch_norm', 'bilinear_tensor_product', 'embedding', 'case', 'cond', 'static_pylayer', 'conv2d',
           'conv2d_transpose', 'conv3d', 'conv3d_transpose', 'data_norm', 'deform_conv2d', 'group_norm',
           'instance_norm', 'layer_norm', 'nce', 'prelu', 'py_func', 'row_conv', 'spectral_norm', 'switch_case',
           'while_loop', 'sparse_embedding', 'sequence_conv', 'sequence_softmax', 'sequence_pool',
           'sequence_first_step', 'sequence_last_step', 'sequence_slice', 'sequence_expand', 'sequence_expand_as',
           'sequence_pad', 'sequence_unpad', 'sequence_reshape', 'sequence_scatter', 'sequence_enumerate']
    missing = [n for n in ref if not callable(getattr(snn, n, None))]
    assert not missing, missing
