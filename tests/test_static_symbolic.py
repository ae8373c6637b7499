"""Symbolic dynamic dims of static Programs (static/symbolic.py; reference: paddle/pir/include/dialect/
shape/utils/dim_expr.h).  Integer constants that happen to be multiples of a carrier extent are
never re-specialised; shape arithmetic on dynamic dims is recorded as DimExprs and evaluated with
the fed extents — also after int() drops the SymInt type."""
import numpy as np
import pytest
import torch

import paddle
from paddle import static
from paddle.static import program as P
from paddle.static import symbolic as S


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def test_symint_arithmetic_builds_expressions():
    b = S.SymInt(P.SENTINELS[0], S.Sym(0))
    s = S.SymInt(P.SENTINELS[1], S.Sym(1))
    e = (b * s * 4) // 2 + 3 - b % 5
    assert isinstance(e, S.SymInt)
    assert int(e) == (P.SENTINELS[0] * P.SENTINELS[1] * 4) // 2 + 3 - P.SENTINELS[0] % 5
    assert e.expr.eval({0: 6, 1: 10}) == (6 * 10 * 4) // 2 + 3 - 6 % 5
    assert (-b).expr.eval({0: 7}) == -7
    assert S.sym_max(b, 9).expr.eval({0: 3}) == 9
    assert 2 * 3 == 6 and not isinstance(b * 0 + 5 - b * 0, bool)
    # decoding a carrier-valued extent (output of torch's shape inference)
    d = S.decode_extent(P.SENTINELS[0] * P.SENTINELS[1] * 12, P.SENTINELS)
    assert d.eval({0: 2, 1: 3}) == 72
    assert S.decode_extent(4096, P.SENTINELS) is None


def test_constant_multiple_of_carrier_is_not_respecialised(static_mode):
    """The round-5 failure mode: a recorded integer constant divisible by a carrier prime was
    silently rewritten to the fed batch size times its cofactor."""
    big = 2 * P.SENTINELS[0]
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 4], 'float32')
        y = x + big                      # recorded op, plain-int argument
        k = paddle.full([2], big, 'int64')  # no static input: a captured constant
        z = paddle.reshape(x, [-1, 2])   # dynamic reshape still works
    exe = static.Executor(paddle.CPUPlace())
    for B in (3, 5):
        xv = np.arange(B * 4, dtype='float32').reshape(B, 4)
        yv, kv, zv = exe.run(main, feed={'x': xv}, fetch_list=[y, k, z])
        np.testing.assert_allclose(yv, xv + big)
        np.testing.assert_array_equal(kv, [big, big])
        assert zv.shape == (B * 2, 2)


def test_shape_arithmetic_recorded_as_expressions(static_mode):
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, None, 4], 'float32')
        xt = x._t
        shp = xt.shape
        assert isinstance(shp[0], S.SymInt) and isinstance(shp[1], S.SymInt) and not isinstance(shp[2], S.SymInt)
        n = shp[0] * shp[1]
        from paddle.core.tensor import _wrap
        flat = _wrap(xt.reshape(n, shp[2]))
        half = _wrap(torch.zeros(int(n // 2 + 1)))   # int() drops the type: the value table keeps it
        rows = _wrap(torch.arange(shp[1]))           # factory op of a dynamic extent
    exe = static.Executor(paddle.CPUPlace())
    for B, T in ((2, 3), (4, 5)):
        xv = np.random.RandomState(0).randn(B, T, 4).astype('float32')
        fv, hv, rv = exe.run(main, feed={'x': xv}, fetch_list=[flat, half, rows])
        np.testing.assert_allclose(fv, xv.reshape(B * T, 4))
        assert hv.shape == ((B * T) // 2 + 1,)
        np.testing.assert_array_equal(rv, np.arange(T))


def test_ernie_static_program_variable_batch_and_sequence(static_mode):
    """A whole model program (ERNIE-tiny) runs at several batch sizes and sequence lengths."""
    from paddle.models import ernie_config, ErnieForSequenceClassification
    paddle.seed(3)
    cfg = ernie_config('ernie-tiny', hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        ids = static.data('ids', [None, None], 'int64')
        model = ErnieForSequenceClassification(cfg, num_classes=3)
        model.eval()
        logits = model(ids)
    exe = static.Executor(paddle.CPUPlace())
    exe.run(startup)
    rng = np.random.RandomState(0)
    for B, T in ((2, 8), (5, 16), (3, 11)):
        x = rng.randint(1, cfg.vocab_size, size=(B, T)).astype('int64')
        out, = exe.run(main, feed={'ids': x}, fetch_list=[logits])
        assert out.shape == (B, 3)
        paddle.disable_static()
        try:
            ref = model(paddle.to_tensor(x)).numpy()
        finally:
            paddle.enable_static()
        np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-5)


def test_saved_program_keeps_dim_expressions(static_mode, tmp_path):
    """save_inference_model / load_inference_model round trip keeps the SymInt expressions."""
    main, startup = static.Program(), static.Program()
    with static.program_guard(main, startup):
        x = static.data('x', [None, 6], 'float32')
        xt = x._t
        from paddle.core.tensor import _wrap
        y = _wrap(xt.reshape(xt.shape[0] * 2, 3) * 2.0 + 2 * P.SENTINELS[0])
    exe = static.Executor(paddle.CPUPlace())
    import os
    os.environ['FLAGS_pa_pdmodel'] = '0'  # this framework's own program format
    try:
        static.save_inference_model(str(tmp_path / 'm'), [x], [y], exe, program=main)
        prog, feeds, fetches = static.load_inference_model(str(tmp_path / 'm'), exe)
    finally:
        os.environ.pop('FLAGS_pa_pdmodel')
    assert prog._symbolic
    for B in (1, 4):
        xv = np.random.RandomState(B).randn(B, 6).astype('float32')
        out, = exe.run(prog, feed={feeds[0]: xv}, fetch_list=fetches)
        np.testing.assert_allclose(out, xv.reshape(B * 2, 3) * 2.0 + 2 * P.SENTINELS[0], rtol=1e-6)
