"""paddle.static.quantization: post-training quantisation of a saved inference model (every
calibration algo), the saved int8 model reloaded by load_inference_model / the Predictor, and
quantisation-aware training (quant_aware -> train -> convert).  CPU: the int8 nodes run their
composite (the GPU test of the int8 MFMA path is tests/test_hip_matmul.py / test_hip_quant.py)."""
import os

import numpy as np
import pytest

import paddle
from paddle import static
from paddle.static import quantization as Q


def _mlp_model(tmp_path):
    paddle.set_device('cpu')
    paddle.seed(3)
    paddle.enable_static()
    try:
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data('x', [None, 64], 'float32')
            h = static.nn.fc(x, 128, activation='relu')
            y = static.nn.fc(h, 16)
        exe = static.Executor(paddle.CPUPlace())
        prefix = os.path.join(str(tmp_path), 'fp32', 'mlp')
        static.save_inference_model(prefix, [x], [y], exe, program=main)
    finally:
        paddle.disable_static()
    return prefix, exe


def _samples(n=64, seed=0):
    rng = np.random.RandomState(seed)
    def gen():
        for _ in range(n):
            yield (rng.randn(64).astype('float32'),)
    return gen


@pytest.mark.parametrize('algo', ['abs_max', 'avg', 'hist', 'KL', 'mse', 'min_max'])
def test_ptq_saved_model_roundtrip(tmp_path, algo):
    prefix, exe = _mlp_model(tmp_path)
    paddle.enable_static()
    try:
        prog, feeds, fetch = static.load_inference_model(prefix, exe)
        xs = np.random.RandomState(7).randn(8, 64).astype('float32')
        ref = exe.run(prog, feed={feeds[0]: xs}, fetch_list=fetch)[0]
        ptq = Q.PostTrainingQuantization(exe, os.path.dirname(prefix), sample_generator=_samples(), batch_size=16,
                                         batch_nums=4, algo=algo, quantizable_op_type=['mul', 'matmul_v2'])
        qprog = ptq.quantize()
        kinds = [getattr(n.target, '__name__', '') for n in qprog.nodes]
        assert kinds.count('quant_linear') == 2, kinds
        out = exe.run(qprog, feed={feeds[0]: xs}, fetch_list=qprog._fetch_vars)[0]
        rel = np.abs(out - ref).max() / np.abs(ref).max()
        # abs-max style thresholds keep every value; KL / hist / mse / avg clip the tail on purpose
        assert rel < (0.03 if algo in ('abs_max', 'min_max') else 0.12), (algo, rel)
        saved = ptq.save_quantized_model(os.path.join(str(tmp_path), 'int8') + os.sep)
        prog2, feeds2, fetch2 = static.load_inference_model(saved, exe)
        out2 = exe.run(prog2, feed={feeds2[0]: xs}, fetch_list=fetch2)[0]
        np.testing.assert_allclose(out2, out, rtol=1e-5, atol=1e-5)
    finally:
        paddle.disable_static()
    from paddle import inference as I
    pred = I.create_predictor(I.Config(saved + '.pdmodel', saved + '.pdiparams'))
    np.testing.assert_allclose(pred.run([paddle.to_tensor(xs)])[0].numpy(), out, rtol=1e-5, atol=1e-5)


def test_ptq_not_frozen_keeps_fake_quant(tmp_path):
    prefix, exe = _mlp_model(tmp_path)
    paddle.enable_static()
    try:
        prog, feeds, fetch = static.load_inference_model(prefix, exe)
        xs = np.random.RandomState(7).randn(8, 64).astype('float32')
        ref = exe.run(prog, feed={feeds[0]: xs}, fetch_list=fetch)[0]
        q = Q.PostTrainingQuantization(exe, os.path.dirname(prefix), sample_generator=_samples(), batch_size=16,
                                       batch_nums=2, algo='abs_max', freeze_model=False).quantize()
        names = [getattr(n.target, '__name__', '') for n in q.nodes]
        assert names.count('fake_quant_dequant') == 2
        out = exe.run(q, feed={feeds[0]: xs}, fetch_list=q._fetch_vars)[0]
        assert np.abs(out - ref).max() / np.abs(ref).max() < 0.05
    finally:
        paddle.disable_static()


def test_quant_aware_training_then_convert():
    paddle.set_device('cpu')
    paddle.seed(4)
    paddle.enable_static()
    try:
        main, startup = static.Program(), static.Program()
        with static.program_guard(main, startup):
            x = static.data('x', [None, 32], 'float32')
            lab = static.data('lab', [None], 'int64')
            h = static.nn.fc(x, 64, activation='relu')
            logits = static.nn.fc(h, 4)
            loss = paddle.nn.functional.cross_entropy(logits, lab)
            paddle.optimizer.Adam(learning_rate=1e-2).minimize(loss)
        Q.quant_aware(main, paddle.CPUPlace())
        exe = static.Executor(paddle.CPUPlace())
        rng = np.random.RandomState(0)
        xs = rng.randn(64, 32).astype('float32')
        ys = (xs[:, :4].argmax(1)).astype('int64')
        losses = [float(exe.run(main, feed={'x': xs, 'lab': ys}, fetch_list=[loss])[0]) for _ in range(30)]
        assert losses[-1] < losses[0] * 0.6, losses
        test = main.clone(for_test=True)
        fq = exe.run(test, feed={'x': xs, 'lab': ys}, fetch_list=[logits])[0]
        Q.convert(test, paddle.CPUPlace())
        names = [getattr(n.target, '__name__', '') for n in test.nodes]
        assert names.count('quant_linear') == 2 and 'fq_activation' not in names, names
        q = exe.run(test, feed={'x': xs, 'lab': ys}, fetch_list=[logits])[0]
        assert np.abs(q - fq).max() / np.abs(fq).max() < 0.02
        assert (q.argmax(1) == ys).mean() > 0.8
    finally:
        paddle.disable_static()
