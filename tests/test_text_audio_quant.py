"""paddle.text (viterbi), paddle.audio (features, wav IO), paddle.quantization (QAT/PTQ/convert),
paddle.fft/signal/distribution smoke."""
import itertools
import os

import numpy as np

import paddle


def test_viterbi_matches_bruteforce():
    rng = np.random.RandomState(0)
    B, L, T = 3, 4, 4
    pot = rng.randn(B, L, T).astype('float32')
    tr = rng.randn(T, T).astype('float32')
    lens = np.array([4, 2, 3])
    s, p = paddle.text.viterbi_decode(paddle.to_tensor(pot), paddle.to_tensor(tr), paddle.to_tensor(lens))
    for b in range(B):
        best = None
        for seq in itertools.product(range(T), repeat=int(lens[b])):
            sc = pot[b, 0, seq[0]] + tr[-1, seq[0]] + tr[seq[-1], -2] + sum(
                tr[seq[i - 1], seq[i]] + pot[b, i, seq[i]] for i in range(1, lens[b]))
            if best is None or sc > best[0]:
                best = (sc, seq)
        assert abs(best[0] - s.numpy()[b]) < 1e-4
        assert list(best[1]) == p.numpy()[b][:lens[b]].tolist()


def test_audio_features_and_io(tmp_path):
    x = paddle.to_tensor(np.random.randn(2, 8000).astype('float32'))
    assert paddle.audio.features.MFCC(sr=8000, n_mfcc=13)(x).shape[:2] == [2, 13]
    fb = paddle.audio.functional.compute_fbank_matrix(8000, 512, n_mels=40)
    assert fb.shape == [40, 257] and float(fb.min()) >= 0
    assert abs(paddle.audio.functional.mel_to_hz(paddle.audio.functional.hz_to_mel(440.0)) - 440.0) < 1e-6
    p = str(tmp_path / 'a.wav')
    paddle.audio.save(p, x[:1] * 0.1, 8000)
    w, sr = paddle.audio.load(p)
    assert sr == 8000 and w.shape == [1, 8000]
    np.testing.assert_allclose(w.numpy(), x[:1].numpy() * 0.1, atol=1e-3)


def test_qat_ptq_convert():
    from paddle.quantization import QAT, PTQ, QuantConfig
    from paddle.quantization.quanters import FakeQuanterWithAbsMaxObserver
    from paddle.quantization.observers import AbsmaxObserver
    paddle.seed(0)
    net = paddle.nn.Sequential(paddle.nn.Linear(8, 16), paddle.nn.ReLU(), paddle.nn.Linear(16, 4))
    q = FakeQuanterWithAbsMaxObserver(moving_rate=0.9)
    qat = QAT(QuantConfig(activation=q, weight=q))
    qnet = qat.quantize(net)
    x = paddle.randn([32, 8]).clip(-2.5, 2.5)  # inside the calibrated range (abs-max clips outliers)
    for _ in range(40):  # moving-average abs-max scales start at accum=state=1 and need to warm up
        qnet(paddle.randn([32, 8]))
    out = qnet(x)
    out.sum().backward()
    assert qnet[0].weight.grad is not None
    ref = net(x)
    assert float((out - ref).abs().max()) < 0.1 * float(ref.abs().max()) + 0.05
    ptq = PTQ(QuantConfig(activation=AbsmaxObserver(), weight=None))
    pnet = ptq.quantize(net)
    for _ in range(3):
        pnet(paddle.randn([32, 8]))
    pnet(x)
    frozen = ptq.convert(pnet)
    y = frozen(x)
    assert float((y - ref).abs().max()) < 0.1 * float(ref.abs().max()) + 0.05
    f8 = ptq.convert(pnet, to_fp8=True)
    y8 = f8(x)
    assert float((y8 - ref).abs().max()) < 0.15 * float(ref.abs().max()) + 0.05


def test_fft_signal_distribution():
    x = np.random.rand(2, 64).astype('float32')
    np.testing.assert_allclose(paddle.fft.rfft(paddle.to_tensor(x)).numpy(), np.fft.rfft(x), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(paddle.fft.fftshift(paddle.to_tensor(x)).numpy(), np.fft.fftshift(x))
    w = paddle.to_tensor(np.hanning(16).astype('float32'))
    s = paddle.signal.stft(paddle.to_tensor(x), 16, 4, window=w)
    r = paddle.signal.istft(s, 16, 4, window=w, length=64)
    np.testing.assert_allclose(r.numpy(), x, atol=1e-5)
    from paddle.distribution import Normal, Categorical, kl_divergence, Beta, Dirichlet
    n = Normal(paddle.to_tensor([0.0]), paddle.to_tensor([1.0]))
    assert abs(float(n.log_prob(paddle.to_tensor([0.0]))) + 0.9189385) < 1e-5
    assert abs(float(kl_divergence(n, Normal(paddle.to_tensor([1.0]), paddle.to_tensor([1.0])))) - 0.5) < 1e-6
    c = Categorical(paddle.to_tensor([1.0, 1.0, 2.0]))
    assert abs(float(c.probs(paddle.to_tensor([2]))) - 0.5) < 1e-6
    assert Beta(2.0, 3.0).sample([5]).shape == [5]
    assert Dirichlet(paddle.ones([3])).sample([2]).shape == [2, 3]
    _ = os
