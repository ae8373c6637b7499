"""Autograd, nn layers, optimizers, checkpoints (CPU)."""
import os

import numpy as np
import pytest
import torch

import paddle
import paddle.nn as nn
import paddle.nn.functional as F


def test_backward_and_grad():
    x = paddle.to_tensor([1.0, 2.0, 3.0], stop_gradient=False)
    y = (x ** 2).sum()
    y.backward()
    np.testing.assert_allclose(x.grad.numpy(), [2, 4, 6])
    x.clear_grad()
    z = paddle.exp(x).mean()
    (g,) = paddle.grad([z], [x], create_graph=True)
    np.testing.assert_allclose(g.numpy(), np.exp([1, 2, 3]) / 3, rtol=1e-6)
    with paddle.no_grad():
        w = x * 2
    assert w.stop_gradient


def test_pylayer():
    class Cube(paddle.autograd.PyLayer):
        @staticmethod
        def forward(ctx, x, k=3):
            ctx.save_for_backward(x)
            ctx.k = k
            return x ** k

        @staticmethod
        def backward(ctx, dy):
            x, = ctx.saved_tensor()
            return dy * ctx.k * x ** (ctx.k - 1)

    x = paddle.to_tensor([2.0], stop_gradient=False)
    y = Cube.apply(x)
    y.backward()
    np.testing.assert_allclose(x.grad.numpy(), [12.0])


def test_jacobian_hessian():
    x = paddle.to_tensor([1.0, 2.0], stop_gradient=False)
    y = x * x
    J = paddle.autograd.jacobian(y, x)
    np.testing.assert_allclose(J[:, :].numpy() if hasattr(J[:, :], 'numpy') else J.numpy(), np.diag([2., 4.]))
    z = (x ** 3).sum()
    H = paddle.autograd.hessian(z, x)
    np.testing.assert_allclose(H.numpy(), np.diag([6., 12.]))


def test_layer_basics_and_state_dict(tmp_path):
    class Net(nn.Layer):
        def __init__(self):
            super().__init__()
            self.fc1 = nn.Linear(4, 8)
            self.bn = nn.BatchNorm1D(8)
            self.fc2 = nn.Linear(8, 2, bias_attr=False)

        def forward(self, x):
            return self.fc2(F.relu(self.bn(self.fc1(x))))

    net = Net()
    sd = net.state_dict()
    assert list(sd.keys()) == ['fc1.weight', 'fc1.bias', 'bn.weight', 'bn.bias', 'bn._mean', 'bn._variance',
                               'fc2.weight']
    assert net.fc1.weight.shape == [4, 8]
    assert len(net.parameters()) == 5
    out = net(paddle.randn([3, 4]))
    assert out.shape == [3, 2]
    path = str(tmp_path / 'net.pdparams')
    paddle.save(net.state_dict(), path)
    net2 = Net()
    net2.set_state_dict(paddle.load(path))
    for (k, a), (_, b) in zip(net.state_dict().items(), net2.state_dict().items()):
        np.testing.assert_allclose(a.numpy(), b.numpy(), err_msg=k)
    net.eval()
    assert not net.bn.training


def test_save_load_formats(tmp_path):
    obj = {'a': paddle.to_tensor([1., 2.]), 'b': [paddle.ones([2]).astype('bfloat16'), 3], 'c': 'str'}
    p = str(tmp_path / 'x.pdparams')
    paddle.save(obj, p)
    r = paddle.load(p)
    np.testing.assert_allclose(r['a'].numpy(), [1, 2])
    assert r['b'][0].dtype == paddle.bfloat16 and r['b'][1] == 3 and r['c'] == 'str'
    r2 = paddle.load(p, return_numpy=True)
    assert isinstance(r2['a'], np.ndarray)


def test_restricted_unpickler_refuses_code(tmp_path):
    import pickle

    class Evil:
        def __reduce__(self):
            return (os.system, ('echo pwned',))
    p = str(tmp_path / 'evil.pdparams')
    with open(p, 'wb') as f:
        pickle.dump({'x': Evil()}, f)
    with pytest.raises(pickle.UnpicklingError):
        paddle.load(p)


@pytest.mark.parametrize("opt_name", ['SGD', 'Momentum', 'Adam', 'AdamW', 'RMSProp', 'Adagrad', 'Adamax', 'Lamb',
                                      'Adadelta', 'NAdam', 'RAdam'])
def test_optimizers_decrease_loss(opt_name):
    paddle.seed(1)
    lin = nn.Linear(8, 1)
    X = paddle.randn([64, 8])
    Y = X.sum(axis=1, keepdim=True)
    kw = {'learning_rate': 0.05 if opt_name not in ('Adadelta',) else 1.0, 'parameters': lin.parameters()}
    opt = getattr(paddle.optimizer, opt_name)(**kw)
    l0 = None
    for _ in range(30):
        loss = F.mse_loss(lin(X), Y)
        if l0 is None:
            l0 = float(loss)
        loss.backward()
        opt.step()
        opt.clear_grad()
    assert float(loss) < l0, (opt_name, l0, float(loss))


def test_adam_matches_reference_formula():
    p0 = np.array([1.0, -2.0], dtype='float32')
    g = np.array([0.5, 0.1], dtype='float32')
    w = paddle.create_parameter([2], 'float32', default_initializer=nn.initializer.Assign(p0))
    opt = paddle.optimizer.Adam(learning_rate=0.1, parameters=[w])
    w.grad = paddle.to_tensor(g)
    opt.step()
    m = 0.1 * g
    v = 0.001 * g * g
    lr = 0.1 * np.sqrt(1 - 0.999) / (1 - 0.9)
    ref = p0 - lr * m / (np.sqrt(v) + 1e-8 * np.sqrt(1 - 0.999))
    np.testing.assert_allclose(w.numpy(), ref, rtol=1e-5)


def test_optimizer_state_dict_roundtrip(tmp_path):
    lin = nn.Linear(3, 3)
    opt = paddle.optimizer.AdamW(learning_rate=paddle.optimizer.lr.StepDecay(0.1, 2), parameters=lin.parameters())
    lin(paddle.randn([2, 3])).sum().backward()
    opt.step()
    sd = opt.state_dict()
    assert any(k.endswith('_moment1_0') for k in sd)
    p = str(tmp_path / 'o.pdopt')
    paddle.save(sd, p)
    opt2 = paddle.optimizer.AdamW(learning_rate=paddle.optimizer.lr.StepDecay(0.1, 2), parameters=lin.parameters())
    opt2.set_state_dict(paddle.load(p))
    k = [k for k in sd if k.endswith('_moment1_0')][0]
    pn = k[:-len('_moment1_0')]
    np.testing.assert_allclose(opt2._accumulators['moment1'][pn].numpy(), sd[k].numpy())


def test_lr_schedulers():
    s = paddle.optimizer.lr.CosineAnnealingDecay(1.0, T_max=10)
    vals = []
    for _ in range(10):
        vals.append(s())
        s.step()
    assert vals[0] == 1.0 and vals[-1] < 0.1
    w = paddle.optimizer.lr.LinearWarmup(0.5, 4, 0.0, 0.5)
    seq = []
    for _ in range(6):
        seq.append(w())
        w.step()
    np.testing.assert_allclose(seq[:5], [0, 0.125, 0.25, 0.375, 0.5])
    pw = paddle.optimizer.lr.PiecewiseDecay([2, 4], [1.0, 0.5, 0.1])
    out = []
    for _ in range(5):
        out.append(pw())
        pw.step()
    assert out == [1.0, 1.0, 0.5, 0.5, 0.1]


def test_grad_clip_global_norm():
    lin = nn.Linear(4, 4)
    opt = paddle.optimizer.SGD(learning_rate=0.0, parameters=lin.parameters(),
                               grad_clip=nn.ClipGradByGlobalNorm(1e-3))
    (lin(paddle.randn([8, 4])) * 100).sum().backward()
    opt.step()
    total = np.sqrt(sum((p.grad.numpy() ** 2).sum() for p in lin.parameters()))
    np.testing.assert_allclose(total, 1e-3, rtol=1e-3)


def test_layers_zoo_forward():
    x = paddle.randn([2, 3, 16, 16])
    assert nn.Conv2D(3, 4, 3, padding=1)(x).shape == [2, 4, 16, 16]
    assert nn.Conv2D(3, 4, 3, stride=2, padding='SAME')(x).shape == [2, 4, 8, 8]
    assert nn.Conv2DTranspose(3, 2, 2, stride=2)(x).shape == [2, 2, 32, 32]
    assert nn.MaxPool2D(2)(x).shape == [2, 3, 8, 8]
    assert nn.AdaptiveAvgPool2D(1)(x).shape == [2, 3, 1, 1]
    assert nn.BatchNorm2D(3)(x).shape == [2, 3, 16, 16]
    assert nn.GroupNorm(1, 3)(x).shape == [2, 3, 16, 16]
    assert nn.Upsample(scale_factor=2)(x).shape == [2, 3, 32, 32]
    seq = paddle.randn([2, 5, 8])
    out, (h, c) = nn.LSTM(8, 16, num_layers=2)(seq)
    assert out.shape == [2, 5, 16] and h.shape == [2, 2, 16]
    out, h = nn.GRU(8, 16, direction='bidirect')(seq)
    assert out.shape == [2, 5, 32]
    enc = nn.TransformerEncoder(nn.TransformerEncoderLayer(8, 2, 16, dropout=0.0), 2)
    assert enc(seq).shape == [2, 5, 8]
    mha = nn.MultiHeadAttention(8, 2)
    assert mha(seq).shape == [2, 5, 8]
    t = nn.Transformer(8, 2, 1, 1, 16, dropout=0.0)
    assert t(seq, seq[:, :3]).shape == [2, 3, 8]
    emb = nn.Embedding(10, 4, padding_idx=0)
    assert emb(paddle.to_tensor([[0, 3]])).shape == [1, 2, 4]
    assert float(emb(paddle.to_tensor([0])).abs().sum()) == 0.0


def test_losses():
    logits = paddle.randn([4, 5])
    lab = paddle.to_tensor([0, 1, 2, 3])
    ref = torch.nn.functional.cross_entropy(logits._t, lab._t)
    np.testing.assert_allclose(float(F.cross_entropy(logits, lab)), float(ref), rtol=1e-5)
    np.testing.assert_allclose(float(nn.CrossEntropyLoss()(logits, lab.unsqueeze(-1))), float(ref), rtol=1e-5)
    soft = F.softmax(paddle.randn([4, 5]))
    assert F.cross_entropy(logits, soft, soft_label=True).shape == []
    assert F.softmax_with_cross_entropy(logits, lab.unsqueeze(-1)).shape == [4, 1]
    assert float(F.mse_loss(logits, logits)) == 0.0


def test_lenet_mnist_shaped_training():
    """Config 1 of BASELINE.json: LeNet dygraph on CPU (synthetic MNIST-shaped data)."""
    from paddle.vision.models import LeNet
    paddle.seed(0)
    model = LeNet()
    opt = paddle.optimizer.Adam(learning_rate=1e-3, parameters=model.parameters())
    x = paddle.randn([64, 1, 28, 28])
    y = paddle.randint(0, 10, [64, 1])
    losses = []
    for _ in range(30):
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < 0.5 * losses[0]
