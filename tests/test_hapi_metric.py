"""hapi Model fit/evaluate/predict/save/load, callbacks, summary, flops, metrics."""
import numpy as np

import paddle
from paddle.io import Dataset
from paddle.metric import Accuracy, Precision, Recall, Auc


class Blobs(Dataset):
    def __init__(self, n=256, seed=0):
        rng = np.random.RandomState(seed)
        self.y = rng.randint(0, 3, n)
        centers = np.eye(3, 10) * 4
        self.x = (centers[self.y] + rng.randn(n, 10)).astype('float32')

    def __getitem__(self, i):
        return self.x[i], np.int64(self.y[i])

    def __len__(self):
        return len(self.y)


def _net():
    return paddle.nn.Sequential(paddle.nn.Linear(10, 32), paddle.nn.ReLU(), paddle.nn.Linear(32, 3))


def test_model_fit_evaluate_predict(tmp_path):
    paddle.seed(0)
    model = paddle.Model(_net(), inputs=[paddle.static.InputSpec([None, 10], 'float32', 'x')])
    opt = paddle.optimizer.Adam(learning_rate=0.01, parameters=model.parameters())
    model.prepare(opt, paddle.nn.CrossEntropyLoss(), Accuracy())
    model.fit(Blobs(), epochs=3, batch_size=32, verbose=0)
    res = model.evaluate(Blobs(128, seed=1), batch_size=64, verbose=0)
    assert res['acc'] > 0.85, res
    preds = model.predict(Blobs(16, seed=2), batch_size=8, stack_outputs=True, verbose=0)
    assert preds[0].shape == (16, 3)
    path = str(tmp_path / 'ckpt' / 'm')
    model.save(path)
    m2 = paddle.Model(_net())
    m2.prepare(paddle.optimizer.Adam(parameters=m2.parameters()), paddle.nn.CrossEntropyLoss(), Accuracy())
    m2.load(path)
    res2 = m2.evaluate(Blobs(128, seed=1), batch_size=64, verbose=0)
    assert abs(res2['acc'] - res['acc']) < 1e-6
    model.save(str(tmp_path / 'infer'), training=False)
    loaded = paddle.jit.load(str(tmp_path / 'infer'))
    x = paddle.to_tensor(Blobs(4, seed=3).x[:4])
    np.testing.assert_allclose(loaded(x).numpy(), model.network(x).numpy(), rtol=1e-5, atol=1e-6)


def test_early_stopping_and_lr_callbacks():
    paddle.seed(1)
    model = paddle.Model(_net())
    sched = paddle.optimizer.lr.StepDecay(0.05, step_size=2, gamma=0.5)
    model.prepare(paddle.optimizer.SGD(learning_rate=sched, parameters=model.parameters()),
                  paddle.nn.CrossEntropyLoss(), Accuracy())
    es = paddle.callbacks.EarlyStopping(monitor='acc', mode='max', patience=0, save_best_model=False)
    model.fit(Blobs(64), eval_data=Blobs(64, seed=1), epochs=5, batch_size=16, verbose=0,
              callbacks=[es, paddle.callbacks.LRScheduler(by_step=True)])
    assert sched.last_epoch > 0


def test_summary_and_flops():
    net = paddle.vision.models.LeNet()
    info = paddle.summary(net, (1, 1, 28, 28))
    assert info['total_params'] == sum(int(np.prod(p.shape)) for p in net.parameters())
    f = paddle.flops(net, [1, 1, 28, 28])
    assert f > 100000


def test_metrics():
    acc = Accuracy(topk=(1, 2))
    pred = paddle.to_tensor([[0.1, 0.7, 0.2], [0.5, 0.3, 0.2], [0.2, 0.3, 0.5]])
    lab = paddle.to_tensor([[1], [1], [0]])
    c = acc.compute(pred, lab)
    acc.update(c)
    top1, top2 = acc.accumulate()
    assert abs(top1 - 1 / 3) < 1e-6 and abs(top2 - 2 / 3) < 1e-6
    p, r = Precision(), Recall()
    preds = np.array([0.9, 0.8, 0.2, 0.6])
    labels = np.array([1, 0, 1, 1])
    p.update(preds, labels)
    r.update(preds, labels)
    assert abs(p.accumulate() - 2 / 3) < 1e-6 and abs(r.accumulate() - 2 / 3) < 1e-6
    auc = Auc()
    auc.update(np.stack([1 - preds, preds], 1), labels)
    assert abs(auc.accumulate() - 1 / 3) < 1e-3  # one of three (pos, neg) pairs ranked correctly
    a = paddle.metric.accuracy(pred, lab, k=1)
    assert abs(float(a) - 1 / 3) < 1e-6
