"""FP8 training path (ops/fp8.py, csrc/fp8_cast.hip, csrc/gemm.hip fp8 kernel): delayed scaling,
fp8 Linear autograd, dygraph fp8_autocast, static.amp use_fp8 (BASELINE config 5: ERNIE static
Executor + AMP-O2 fp8).  CPU tests run the torch mirror of the kernels' math; GPU tests compare
the HIP cast / GEMMs against an fp32 torch reference."""
import numpy as np
import pytest
import torch

import paddle
import paddle.static as static
from paddle.ops import fp8 as F8


def test_recipe_validation():
    r = F8.DelayedScaling(margin=1, fp8_format='hybrid', amax_history_len=8)
    assert r.fwd_dtype == torch.float8_e4m3fn and r.bwd_dtype == torch.float8_e5m2
    assert F8.DelayedScaling(fp8_format='E4M3').bwd_dtype == torch.float8_e4m3fn
    with pytest.raises(ValueError):
        F8.DelayedScaling(fp8_format='E5M2')
    with pytest.raises(ValueError):
        F8.DelayedScaling(amax_history_len=2)


def test_meta_delayed_scaling_cpu():
    m = F8.FP8Meta(torch.float8_e4m3fn, 4, 0, 'cpu')
    x = torch.randn(16, 32).to(torch.bfloat16) * 3
    q, qt, sinv = m.cast(x)
    amax = x.float().abs().max()
    # first call is seeded with the exact amax: scale = 448 / amax
    np.testing.assert_allclose(float(sinv), float(amax) / 448.0, rtol=1e-6)
    assert q.shape == (16, 32) and qt.shape == (32, 16)
    assert torch.equal(q.t().contiguous().view(torch.uint8), qt.view(torch.uint8))
    deq = q.float() * sinv
    assert (deq - x.float()).abs().max() <= amax * 2 ** -3  # e4m3: 3 mantissa bits
    # the current amax lands in slot 0, slot 1 (next call's) is cleared
    assert float(m.hist[0]) == pytest.approx(float(amax))
    x2 = x * 10
    _, _, s2 = m.cast(x2, want_qt=False)
    # scale of call 2 comes from the history (slot 3 = seed, slot 0 = call 1): still amax(x)
    np.testing.assert_allclose(float(s2), float(amax) / 448.0, rtol=1e-6)
    _, _, s3 = m.cast(x2, want_qt=False)
    np.testing.assert_allclose(float(s3), float(x2.float().abs().max()) / 448.0, rtol=1e-5)


def test_margin_and_empty_history():
    m = F8.FP8Meta(torch.float8_e5m2, 4, 2, 'cpu')
    m.calls = 1  # skip the seeding pre-pass: empty history -> unit scale
    _, _, s = m.cast(torch.ones(8, 8, dtype=torch.bfloat16))
    assert float(s) == 1.0
    _, _, s = m.cast(torch.ones(8, 8, dtype=torch.bfloat16))
    np.testing.assert_allclose(float(s), 1.0 / (57344.0 / 4), rtol=1e-6)  # margin 2 -> /4


def test_fp8_linear_grads_cpu():
    torch.manual_seed(0)
    x = torch.randn(64, 32, dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(32, 48, dtype=torch.bfloat16, requires_grad=True)
    b = torch.randn(48, dtype=torch.bfloat16, requires_grad=True)
    st = F8.FP8State(F8.DelayedScaling(), 'cpu')
    y = F8._FP8Linear.apply(x, w, b, st)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = xr @ wr + br
    yr.backward(g.float())
    def rel(a, b_):
        return float((a.float() - b_).norm() / b_.norm())
    assert rel(y.detach(), yr.detach()) < 0.08
    assert rel(x.grad, xr.grad) < 0.15
    assert rel(w.grad, wr.grad) < 0.15
    assert rel(b.grad, br.grad) < 0.02


def test_dygraph_fp8_autocast_cpu():
    paddle.seed(0)
    lin = paddle.nn.Linear(32, 16)
    x = paddle.randn([8, 32])
    ref = lin(x).numpy()
    with paddle.amp.fp8_autocast():
        y = lin(x)
    assert '_fp8_state' in lin.weight.__dict__
    rel = np.linalg.norm(y.astype('float32').numpy() - ref) / np.linalg.norm(ref)
    assert rel < 0.1
    y.astype('float32').sum().backward()
    assert lin.weight.grad is not None and lin.bias.grad is not None


def _ernie_fp8(dev, place, S, B, steps):
    from paddle.models import ernie_config, ErnieForSequenceClassification
    paddle.seed(3)
    cfg = ernie_config('ernie-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        ids = static.data('ids', [None, S], 'int64')
        lab = static.data('lab', [None], 'int64')
        model = ErnieForSequenceClassification(cfg, num_classes=2)
        loss = paddle.nn.functional.cross_entropy(model(ids), lab)
        opt = paddle.optimizer.AdamW(learning_rate=2e-3, parameters=model.parameters())
        opt = static.amp.decorate(opt, level='O2', use_fp8=True,
                                  fp8_recipe=paddle.amp.DelayedScaling(amax_history_len=8))
        opt.minimize(loss)
    exe = static.Executor(place)
    exe.run(startup)
    opt.amp_init(place)
    rng = np.random.RandomState(0)
    x = rng.randint(1, cfg.vocab_size, size=(B, S)).astype('int64')
    y = (x[:, 0] % 2).astype('int64')
    losses = [float(exe.run(main, feed={'ids': x, 'lab': y}, fetch_list=[loss])[0]) for _ in range(steps)]
    return losses, main


def test_ernie_static_fp8_cpu(static_mode):
    """BASELINE config 5 on CPU: ERNIE static Program, Executor, AMP-O2 with fp8 Linears."""
    F8._STATIC_STATES.clear()
    losses, main = _ernie_fp8('cpu', paddle.CPUPlace(), 16, 8, 25)
    assert len(F8._STATIC_STATES) > 0  # the recorded Linears went through the fp8 path
    assert np.isfinite(losses).all(), losses
    assert losses[-1] < losses[0] * 0.6, losses


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("R,C", [(256, 512), (200, 136), (1024, 2048)])
@pytest.mark.parametrize("dtype", [torch.float8_e4m3fn, torch.float8_e5m2])
def test_hip_cast_transpose(R, C, dtype):
    from paddle.ops import _native as N
    assert N._load() is not None, N.load_error
    torch.manual_seed(1)
    x = (torch.randn(R, C, device='cuda') * 5).to(torch.bfloat16)
    m = F8.FP8Meta(dtype, 8, 0, 'cuda')
    q, qt, sinv = m.cast(x)
    torch.cuda.synchronize()
    amax = x.float().abs().max()
    fm = 448.0 if dtype == torch.float8_e4m3fn else 57344.0
    torch.testing.assert_close(sinv.cpu(), (amax / fm).reshape(1).cpu(), rtol=1e-6, atol=0)
    ref = (x.float() * (fm / amax)).clamp(-fm, fm).to(dtype)
    # hardware round-to-nearest-even == torch's cast, bit for bit
    assert torch.equal(q.view(torch.uint8), ref.view(torch.uint8))
    assert torch.equal(qt.view(torch.uint8), ref.t().contiguous().view(torch.uint8))
    assert float(m.hist[0]) == float(amax)
    assert float(m.hist[1]) == 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("R,C", [(128, 128), (384, 1152), (16384, 2048)])
def test_hip_cast_transpose_full_tiles_bitwise(R, C):
    """The persistent and the one-tile full-tile cast kernels == the guarded per-tile kernel, byte
    for byte."""
    from paddle.ops import _native as N
    assert N._load() is not None, N.load_error
    torch.manual_seed(2)
    x = (torch.randn(R, C, device='cuda') * 3).to(torch.bfloat16)
    outs = []
    for full in (2, 1, 0):  # persistent, one tile per block, guarded
        old = N.lib.pa_fp8_set_cast_full(full)
        try:
            m = F8.FP8Meta(torch.float8_e4m3fn, 8, 0, 'cuda')
            q, qt, sinv = m.cast(x)
            torch.cuda.synchronize()
            outs.append((q.view(torch.uint8).clone(), qt.view(torch.uint8).clone(), sinv.clone(), m.hist.clone()))
        finally:
            N.lib.pa_fp8_set_cast_full(old)
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


@pytest.mark.gpu
def test_hip_fp8_linear_vs_fp32():
    from paddle.ops import _native as N
    assert N._load() is not None, N.load_error
    torch.manual_seed(0)
    M, K, Nn = 512, 1024, 768
    x = torch.randn(M, K, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(K, Nn, device='cuda') * 0.03).to(torch.bfloat16).requires_grad_()
    b = torch.randn(Nn, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    st = F8.FP8State(F8.DelayedScaling(), 'cuda')
    g = torch.randn(M, Nn, device='cuda', dtype=torch.bfloat16)
    for _ in range(3):  # history warms up; every step must stay accurate
        x.grad = w.grad = b.grad = None
        y = F8._FP8Linear.apply(x, w, b, st)
        y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_() for t in (x, w, b))
    yr = xr @ wr + br
    yr.backward(g.float())
    def rel(a, b_):
        return float((a.float() - b_).norm() / b_.norm())
    assert rel(y.detach(), yr.detach()) < 0.06
    assert rel(x.grad, xr.grad) < 0.12
    assert rel(w.grad, wr.grad) < 0.12
    assert rel(b.grad, br.grad) < 1e-2  # the bias gradient: exact column sums of dY (from the dY cast)


@pytest.mark.gpu
@pytest.mark.parametrize("R,C", [(512, 768), (32768 // 8, 2304), (256, 128)])
def test_hip_cast_transpose_column_sums(R, C):
    """The dY cast's per-128-row-tile column sums (pa_fp8_cast_transpose_cs) == torch sums of the
    same bf16 tiles, and its q / q^T bytes == the plain cast's."""
    from paddle.ops import _native as N
    assert N._load() is not None, N.load_error
    torch.manual_seed(4)
    x = (torch.randn(R, C, device='cuda') * 2).to(torch.bfloat16)
    cs = torch.empty((R // 128) * C, dtype=torch.float32, device='cuda')
    m1 = F8.FP8Meta(torch.float8_e5m2, 8, 0, 'cuda')
    q1, qt1, s1 = m1.cast(x, colsum=cs)
    assert m1.cs_done
    m0 = F8.FP8Meta(torch.float8_e5m2, 8, 0, 'cuda')
    q0, qt0, s0 = m0.cast(x)
    torch.cuda.synchronize()
    assert torch.equal(q1.view(torch.uint8), q0.view(torch.uint8))
    assert torch.equal(qt1.view(torch.uint8), qt0.view(torch.uint8))
    ref = x.float().reshape(R // 128, 128, C).sum(1).reshape(-1)
    assert torch.allclose(cs, ref, rtol=1e-5, atol=1e-3), (cs - ref).abs().max().item()


@pytest.mark.gpu
def test_hip_fp8_linear_bias_grad_paths_agree():
    """fp8 Linear bias gradient from the dY cast's column sums == the separate column-sum pass."""
    torch.manual_seed(1)
    M, K, Nn = 1024, 256, 384
    x = torch.randn(M, K, device='cuda', dtype=torch.bfloat16, requires_grad=True)
    w = (torch.randn(K, Nn, device='cuda') * 0.05).to(torch.bfloat16).requires_grad_()
    g = torch.randn(M, Nn, device='cuda', dtype=torch.bfloat16)
    got = []
    for flag in (True, False):
        F8.BIAS_FROM_CAST = flag
        try:
            b = torch.zeros(Nn, device='cuda', dtype=torch.bfloat16, requires_grad=True)
            st = F8.FP8State(F8.DelayedScaling(), 'cuda')
            F8._FP8Linear.apply(x, w, b, st).backward(g)
            got.append(b.grad.float().clone())
        finally:
            F8.BIAS_FROM_CAST = True
    assert torch.allclose(got[0], got[1], rtol=1e-2, atol=1e-2), (got[0] - got[1]).abs().max().item()


@pytest.mark.gpu
def test_ernie_static_fp8_gpu(static_mode):
    """BASELINE config 5 on the MI355X: ERNIE static Executor, AMP-O2 + fp8 (HIP cast + fp8 MFMA)."""
    paddle.set_device('gpu')
    try:
        F8._STATIC_STATES.clear()
        losses, main = _ernie_fp8('gpu', paddle.CUDAPlace(0), 128, 16, 25)
        assert len(F8._STATIC_STATES) > 0
        assert np.isfinite(losses).all() and losses[-1] < losses[0] * 0.6, losses
    finally:
        paddle.set_device('cpu')


@pytest.mark.gpu
def test_hip_batched_weight_cast_equals_per_linear_casts():
    """begin_static_step: every static fp8 weight cast in one launch == one cast per weight
    (q, q^T, dequant scale and the amax history, byte for byte), and the Linear consumes it."""
    from paddle.ops import _native as N
    assert N._load() is not None, N.load_error
    torch.manual_seed(5)
    shapes = [(768, 768), (768, 3072), (3072, 768), (256, 128)]
    ws = [(torch.randn(*s, device='cuda') * 0.05).to(torch.bfloat16).requires_grad_() for s in shapes]
    saved = dict(F8._STATIC_STATES)
    F8._STATIC_STATES.clear()
    try:
        rec = F8.DelayedScaling()
        sts = []
        for i, w in enumerate(ws):
            st = F8._static_state(w, rec, key=('t', i))
            st.wref = __import__('weakref').ref(w)
            st.w.cast(w)  # seeds the history (step 0 of a run)
            sts.append(st)
        refs = []
        for st, w in zip(sts, ws):  # the per-Linear cast on a copy of each meta
            m = F8.FP8Meta(st.w.dtype, st.w.L, 0, 'cuda')
            m.hist.copy_(st.w.hist)
            m.cur, m.calls = st.w.cur, st.w.calls
            q, qt, s = m.cast(w)
            refs.append((q.view(torch.uint8), qt.view(torch.uint8), s, m.hist, m.cur))
        F8.begin_static_step()
        torch.cuda.synchronize()
        for st, w, (q, qt, s, h, cur) in zip(sts, ws, refs):
            bq, bqt, bs = st.w.cast_weight(w)
            assert torch.equal(bq.view(torch.uint8), q) and torch.equal(bqt.view(torch.uint8), qt)
            assert torch.equal(bs, s) and torch.equal(st.w.hist, h) and st.w.cur == cur
        x = torch.randn(64, 768, device='cuda', dtype=torch.bfloat16)
        y = F8._FP8Linear.apply(x, ws[0], None, sts[0])
        yr = x.float() @ ws[0].detach().float()
        assert float((y.float() - yr).norm() / yr.norm()) < 0.06
    finally:
        F8._STATIC_STATES.clear()
        F8._STATIC_STATES.update(saved)
