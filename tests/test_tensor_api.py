"""Tensor API numerics vs numpy (reference strategy: test/legacy_test OpTest = numpy forward reference)."""
import numpy as np
import pytest

import paddle


def npt(x):
    return np.asarray(x)


def test_creation():
    assert paddle.zeros([2, 3]).shape == [2, 3]
    assert paddle.ones([2], dtype='int32').dtype == paddle.int32
    np.testing.assert_allclose(npt(paddle.arange(0, 10, 2)), np.arange(0, 10, 2))
    assert paddle.arange(5).dtype == paddle.int64
    assert paddle.arange(0.0, 1.0, 0.25).dtype == paddle.float32
    np.testing.assert_allclose(npt(paddle.linspace(0, 1, 5)), np.linspace(0, 1, 5), rtol=1e-6)
    np.testing.assert_allclose(npt(paddle.eye(3)), np.eye(3))
    np.testing.assert_allclose(npt(paddle.full([2, 2], 7.0)), np.full((2, 2), 7.0))
    t = paddle.to_tensor([1.5, 2.5])
    assert t.dtype == paddle.float32 and t.stop_gradient
    assert paddle.to_tensor(np.array([1, 2], dtype=np.int64)).dtype == paddle.int64
    np.testing.assert_allclose(npt(paddle.tril(paddle.ones([3, 3]))), np.tril(np.ones((3, 3))))
    a, b = paddle.meshgrid(paddle.arange(2), paddle.arange(3))
    assert a.shape == [2, 3]


def test_math_elementwise():
    x = np.random.rand(3, 4).astype('float32') + 0.1
    y = np.random.rand(3, 4).astype('float32') + 0.1
    px, py = paddle.to_tensor(x), paddle.to_tensor(y)
    for name, ref in [('add', np.add), ('subtract', np.subtract), ('multiply', np.multiply),
                      ('divide', np.divide), ('maximum', np.maximum), ('minimum', np.minimum), ('pow', np.power)]:
        np.testing.assert_allclose(npt(getattr(paddle, name)(px, py)), ref(x, y), rtol=1e-5, err_msg=name)
    for name, ref in [('exp', np.exp), ('log', np.log), ('sqrt', np.sqrt), ('sin', np.sin), ('tanh', np.tanh),
                      ('abs', np.abs), ('floor', np.floor), ('rsqrt', lambda v: 1 / np.sqrt(v))]:
        np.testing.assert_allclose(npt(getattr(paddle, name)(px)), ref(x), rtol=1e-5, err_msg=name)
    np.testing.assert_allclose(npt(px + 1), x + 1, rtol=1e-6)
    np.testing.assert_allclose(npt(2 * px - py / 3), 2 * x - y / 3, rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.clip(px, 0.3, 0.6)), np.clip(x, 0.3, 0.6))
    np.testing.assert_allclose(npt(paddle.scale(px, 2.0, 1.0)), x * 2 + 1, rtol=1e-6)
    np.testing.assert_allclose(npt(paddle.mod(paddle.to_tensor([-3, 5]), paddle.to_tensor([2, 3]))), [1, 2])


def test_reductions():
    x = np.random.rand(2, 3, 4).astype('float32')
    p = paddle.to_tensor(x)
    np.testing.assert_allclose(npt(paddle.sum(p)), x.sum(), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.sum(p, axis=[0, 2], keepdim=True)), x.sum((0, 2), keepdims=True), rtol=1e-5)
    np.testing.assert_allclose(npt(p.mean(axis=1)), x.mean(1), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.max(p, axis=-1)), x.max(-1))
    np.testing.assert_allclose(npt(paddle.min(p)), x.min())
    np.testing.assert_allclose(npt(paddle.prod(p, axis=0)), x.prod(0), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.cumsum(p, axis=1)), x.cumsum(1), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.logsumexp(p, axis=-1)), np.log(np.exp(x).sum(-1)), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.std(p, axis=0)), x.std(0, ddof=1), rtol=1e-4)
    np.testing.assert_allclose(npt(paddle.argmax(p, axis=2)), x.argmax(2))
    assert paddle.argmax(p).shape == []
    assert paddle.sum(paddle.to_tensor([True, False, True])).item() == 2
    np.testing.assert_allclose(npt(paddle.median(paddle.to_tensor([3., 1., 2., 4.]))), 2.5)


def test_manipulation():
    x = np.arange(24).reshape(2, 3, 4).astype('float32')
    p = paddle.to_tensor(x)
    assert paddle.reshape(p, [4, -1]).shape == [4, 6]
    assert paddle.reshape(p, [0, -1]).shape == [2, 12]
    np.testing.assert_allclose(npt(paddle.transpose(p, [2, 0, 1])), x.transpose(2, 0, 1))
    np.testing.assert_allclose(npt(paddle.concat([p, p], axis=1)), np.concatenate([x, x], 1))
    np.testing.assert_allclose(npt(paddle.stack([p, p])), np.stack([x, x]))
    parts = paddle.split(p, 2, axis=2)
    assert len(parts) == 2 and parts[0].shape == [2, 3, 2]
    parts = paddle.split(p, [1, -1], axis=1)
    assert parts[1].shape == [2, 2, 4]
    assert paddle.unsqueeze(p, [0, 2]).shape == [1, 2, 1, 3, 4]
    assert paddle.squeeze(paddle.ones([1, 3, 1]), axis=0).shape == [3, 1]
    assert paddle.flatten(p, 1).shape == [2, 12]
    np.testing.assert_allclose(npt(paddle.gather(p, paddle.to_tensor([1, 0]), axis=1)), x[:, [1, 0]])
    idx = np.array([[0, 1], [1, 2]])
    np.testing.assert_allclose(npt(paddle.gather_nd(p, paddle.to_tensor(idx))), x[idx[:, 0], idx[:, 1]])
    np.testing.assert_allclose(npt(paddle.tile(paddle.to_tensor([1, 2]), [2])), [1, 2, 1, 2])
    np.testing.assert_allclose(npt(paddle.expand(paddle.ones([1, 3]), [2, 3])), np.ones((2, 3)))
    np.testing.assert_allclose(npt(paddle.flip(p, [0])), x[::-1])
    np.testing.assert_allclose(npt(paddle.roll(paddle.arange(4), 1)), [3, 0, 1, 2])
    np.testing.assert_allclose(npt(paddle.slice(p, [1, 2], [0, 1], [2, 3])), x[:, 0:2, 1:3])
    np.testing.assert_allclose(npt(paddle.strided_slice(p, [2], [0], [4], [2])), x[:, :, 0:4:2])
    u = paddle.scatter(paddle.zeros([3, 2]), paddle.to_tensor([1]), paddle.ones([1, 2]))
    np.testing.assert_allclose(npt(u), [[0, 0], [1, 1], [0, 0]])
    s = paddle.scatter_nd_add(paddle.zeros([3]), paddle.to_tensor([[1], [1]]), paddle.to_tensor([1., 2.]))
    np.testing.assert_allclose(npt(s), [0, 3, 0])
    np.testing.assert_allclose(npt(paddle.take_along_axis(p, paddle.to_tensor(np.zeros((2, 3, 1), 'int64')), 2)),
                               x[:, :, :1])
    np.testing.assert_allclose(npt(paddle.where(p > 10, p, paddle.zeros_like(p))), np.where(x > 10, x, 0))
    assert paddle.nonzero(paddle.to_tensor([0, 1, 0, 2])).shape == [2, 1]
    vals, idxs = paddle.topk(paddle.to_tensor([1., 5., 3.]), 2)
    np.testing.assert_allclose(npt(vals), [5, 3])
    np.testing.assert_allclose(npt(paddle.unique(paddle.to_tensor([3, 1, 3, 2]))), [1, 2, 3])


def test_indexing():
    x = np.arange(12).reshape(3, 4).astype('float32')
    p = paddle.to_tensor(x)
    np.testing.assert_allclose(npt(p[1]), x[1])
    np.testing.assert_allclose(npt(p[:, 1:3]), x[:, 1:3])
    np.testing.assert_allclose(npt(p[paddle.to_tensor([0, 2])]), x[[0, 2]])
    np.testing.assert_allclose(npt(p[p > 5]), x[x > 5])
    p[0, 0] = 100.0
    assert p[0, 0].item() == 100.0


def test_linalg():
    a = np.random.rand(3, 4).astype('float32')
    b = np.random.rand(4, 5).astype('float32')
    np.testing.assert_allclose(npt(paddle.matmul(paddle.to_tensor(a), paddle.to_tensor(b))), a @ b, rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.matmul(paddle.to_tensor(b), paddle.to_tensor(a), transpose_x=True,
                                                 transpose_y=True)), b.T @ a.T, rtol=1e-5)
    m = np.random.rand(4, 4).astype('float32') + 4 * np.eye(4, dtype='float32')
    np.testing.assert_allclose(npt(paddle.linalg.inv(paddle.to_tensor(m))), np.linalg.inv(m), rtol=1e-4)
    np.testing.assert_allclose(npt(paddle.linalg.det(paddle.to_tensor(m))), np.linalg.det(m), rtol=1e-4)
    np.testing.assert_allclose(npt(paddle.linalg.norm(paddle.to_tensor(a))), np.linalg.norm(a), rtol=1e-5)
    np.testing.assert_allclose(npt(paddle.einsum('ij,jk->ik', paddle.to_tensor(a), paddle.to_tensor(b))), a @ b,
                               rtol=1e-5)


def test_dtypes_and_cast():
    x = paddle.to_tensor([1.7, -2.3])
    assert x.astype('int32').dtype == paddle.int32
    assert x.cast(paddle.bfloat16).dtype == paddle.bfloat16
    assert paddle.get_default_dtype() == 'float32'
    assert paddle.finfo(paddle.float16).max == 65504.0
    assert x.numpy().dtype == np.float32
    assert x.astype('bfloat16').numpy().dtype == np.uint16  # paddle's bf16 numpy convention


def test_onnx_export_emits_model_proto(tmp_path):
    """paddle.onnx.export writes an ONNX ModelProto (no onnx package: decoded by paddle.onnx.inspect)."""
    import paddle
    from paddle.static import InputSpec

    class Net(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.conv = paddle.nn.Conv2D(3, 4, 3, padding=1)
            self.fc = paddle.nn.Linear(4 * 8 * 8, 5)
            self.ln = paddle.nn.LayerNorm(5)

        def forward(self, x):
            h = paddle.nn.functional.relu(self.conv(x)).flatten(1)
            return paddle.nn.functional.softmax(self.ln(self.fc(h)), -1)

    f = paddle.onnx.export(Net(), str(tmp_path / 'net'), input_spec=[InputSpec([None, 3, 8, 8], 'float32', 'img')])
    assert f.endswith('net.onnx')
    info = paddle.onnx.inspect(f)
    assert info['opset'] >= 13 and info['inputs'] == ['img']
    for op in ('Conv', 'Relu', 'Gemm', 'Softmax'):
        assert op in info['ops'], info['ops']


def test_linalg_ormqr_reference_docstring():
    """reference tensor/linalg.py:5075-5083 example values."""
    import numpy as np
    import paddle
    x = paddle.to_tensor([[-114.6, 10.9, 1.1], [-0.304, 38.07, 69.38], [-0.45, -0.17, 62]])
    tau = paddle.to_tensor([1.55, 1.94, 3.0])
    out = paddle.linalg.ormqr(x, tau, x)
    ref = np.array([[63.82712936, -13.82312393, -116.28614044], [-53.65926361, -28.15783691, -70.42700958],
                    [-79.54292297, 24.00182915, -41.34253311]])
    np.testing.assert_allclose(out.numpy(), ref, rtol=1e-4, atol=1e-3)
    # transpose / right multiplication agree with the explicit Q from householder_product
    q = paddle.linalg.householder_product(x, tau).numpy()
    y = np.random.RandomState(0).randn(3, 3).astype('float32')
    np.testing.assert_allclose(paddle.linalg.ormqr(x, tau, paddle.to_tensor(y), transpose=True).numpy(), q.T @ y,
                               rtol=1e-4, atol=1e-3)
    np.testing.assert_allclose(paddle.linalg.ormqr(x, tau, paddle.to_tensor(y), left=False).numpy(), y @ q,
                               rtol=1e-4, atol=1e-3)
