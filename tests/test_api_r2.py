"""Round-2 API additions: paddle.nn.quant (weight-only int8/int4, LLM.int8), incubate.autograd
(Jacobian / Hessian / forward_grad), fused_bias_dropout_residual_layer_norm, ASP
add_supported_layer, paddle.hub / paddle.callbacks modules, incubate LBFGS."""
import numpy as np
import pytest

import paddle
import paddle.nn.functional as F


@pytest.mark.parametrize('algo,group', [('weight_only_int8', -1), ('weight_only_int8', 64), ('weight_only_int4', -1),
                                        ('weight_only_int4', 128), ('llm.int8', -1)])
def test_weight_quantize_roundtrip(algo, group):
    from paddle.nn.quant import weight_quantize, weight_dequantize
    rs = np.random.RandomState(0)
    w = rs.randn(256, 48).astype('float32')
    q, s = weight_quantize(paddle.to_tensor(w), algo=algo, group_size=group)
    k, n = w.shape
    assert q.shape == ([n, k // 2] if algo == 'weight_only_int4' else [n, k])
    assert s.shape == ([n] if group == -1 else [k // group, n])
    d = weight_dequantize(q, s, algo=algo, out_dtype='float32', group_size=group).numpy()
    qmax = 7 if algo == 'weight_only_int4' else 127
    step = np.abs(w).max() / qmax
    assert d.shape == w.shape and np.abs(d - w).max() <= 0.5 * step + 1e-6


def test_weight_only_linear_and_llm_int8():
    from paddle.nn.quant import weight_quantize, weight_dequantize, weight_only_linear, llm_int8_linear
    rs = np.random.RandomState(1)
    w = rs.randn(64, 32).astype('float32')
    x = rs.randn(6, 64).astype('float32')
    b = rs.randn(32).astype('float32')
    q, s = weight_quantize(paddle.to_tensor(w))
    wd = weight_dequantize(q, s, out_dtype='float32').numpy()
    y = weight_only_linear(paddle.to_tensor(x), q, bias=paddle.to_tensor(b), weight_scale=s).numpy()
    np.testing.assert_allclose(y, x @ wd + b, rtol=1e-5, atol=1e-4)
    x[:, 5] = 30.0  # outlier feature column: computed in floating point
    y8 = llm_int8_linear(paddle.to_tensor(x), q, weight_scale=s, threshold=6.0).numpy()
    ref = x @ wd
    assert np.abs(y8 - ref).max() < 0.02 * np.abs(ref).max()


def test_stub_is_identity():
    from paddle.nn.quant import Stub
    x = paddle.randn([2, 3])
    assert (Stub()(x) == x).all()


def test_fused_bias_dropout_residual_layer_norm():
    import paddle.incubate.nn.functional as IF
    rs = np.random.RandomState(2)
    x, r = rs.randn(2, 5, 16).astype('float32'), rs.randn(2, 5, 16).astype('float32')
    b, g, beta = rs.randn(16).astype('float32'), rs.rand(16).astype('float32'), rs.randn(16).astype('float32')
    t = paddle.to_tensor
    y = IF.fused_bias_dropout_residual_layer_norm(t(x), t(r), t(b), t(g), t(beta), dropout_rate=0.0).numpy()
    h = x + b + r
    ref = (h - h.mean(-1, keepdims=True)) / np.sqrt(h.var(-1, keepdims=True) + 1e-5) * g + beta
    np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-4)
    paddle.seed(0)
    yd = IF.fused_bias_dropout_residual_layer_norm(t(x), t(r), t(b), t(g), t(beta), dropout_rate=0.5).numpy()
    assert yd.shape == ref.shape and not np.allclose(yd, ref)
    layer = paddle.incubate.nn.FusedBiasDropoutResidualLayerNorm(16, dropout_rate=0.0)
    assert layer(t(x), t(r)).shape == [2, 5, 16]


def test_incubate_autograd():
    from paddle.incubate import autograd as A
    x = paddle.to_tensor([1.0, 2.0, 3.0])
    J = A.Jacobian(lambda x: x * x, x)
    np.testing.assert_allclose(J[:].numpy(), np.diag([2.0, 4.0, 6.0]))
    H = A.Hessian(lambda x: (x ** 3).sum(), x)
    np.testing.assert_allclose(H[:].numpy(), np.diag([6.0, 12.0, 18.0]))
    Jb = A.Jacobian(lambda x: x * x, paddle.to_tensor([[1.0, 2.0], [3.0, 4.0]]), is_batched=True)
    np.testing.assert_allclose(Jb[:].numpy(), np.stack([np.diag([2.0, 4.0]), np.diag([6.0, 8.0])]))
    x.stop_gradient = False
    y = paddle.sin(x) * 2
    np.testing.assert_allclose(A.forward_grad(y, x).numpy(), 2 * np.cos([1.0, 2.0, 3.0]), rtol=1e-6)
    np.testing.assert_allclose(A.grad(y.sum(), x).numpy(), 2 * np.cos([1.0, 2.0, 3.0]), rtol=1e-6)


def test_asp_add_supported_layer_custom_pruning():
    from paddle.incubate import asp

    class MyLayer(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.w = self.create_parameter([8, 8])

        def forward(self, x):
            return x @ self.w

    seen = []

    def prune(w, m, n, algo, name):
        seen.append(name)
        mask = (np.arange(w.size).reshape(w.shape) % 2 == 0).astype(w.dtype)
        return w * mask, mask

    asp.add_supported_layer(MyLayer, prune)
    model = MyLayer()
    masks = asp.prune_model(model)
    assert seen == ['w'] and 'w' in masks
    assert (model.w.numpy().reshape(-1)[1::2] == 0).all()


def test_module_aliases():
    import paddle.callbacks
    import paddle.hub
    from paddle.incubate.optimizer import LBFGS
    assert paddle.callbacks.EarlyStopping is paddle.hapi.callbacks.EarlyStopping
    assert callable(paddle.hub.list) and LBFGS is paddle.optimizer.LBFGS
    assert callable(F.flash_attn_varlen_qkvpacked)


def test_fleet_data_generators_and_util(capsys):
    import io
    import sys
    import paddle.distributed.fleet as fleet

    class Words(fleet.MultiSlotDataGenerator):
        def generate_sample(self, line):
            def it():
                toks = [int(t) for t in line.split()]
                yield [('words', toks[:-1]), ('label', [toks[-1]])]
            return it

    class Str(fleet.MultiSlotStringDataGenerator):
        def generate_sample(self, line):
            def it():
                yield [('q', line.split()), ('t', ['x'])]
            return it

    old = sys.stdin
    try:
        sys.stdin = io.StringIO("1 2 3 0\n7 1\n")
        Words().run_from_stdin()
        sys.stdin = io.StringIO("a b\n")
        Str().run_from_stdin()
    finally:
        sys.stdin = old
    out = capsys.readouterr().out.splitlines()
    assert out == ['3 1 2 3 1 0', '1 7 1 1', '2 a b 1 x']
    with pytest.raises(ValueError):
        Words()._gen_str([('words', [])])
    assert fleet.util.get_file_shard(['a', 'b', 'c']) == ['a', 'b', 'c']  # one worker
    assert isinstance(fleet.fleet, fleet.Fleet)


def test_hdfs_client_without_hadoop(tmp_path):
    from paddle.distributed.fleet.utils import HDFSClient, ExecuteError
    c = HDFSClient(str(tmp_path), {'fs.default.name': 'hdfs://x'})
    with pytest.raises(ExecuteError):
        c.is_exist('/a')
