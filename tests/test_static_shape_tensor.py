"""Static-mode shape tensors (reference: paddle.shape -> a shape op whose value is known only at run
time; reshape2's ShapeTensor / ShapeTensorList inputs): paddle.shape of a Variable with a dynamic
batch dim is a recorded node, and reshape accepts it (or its elements) as the target shape."""
import numpy as np
import pytest

import paddle


@pytest.fixture
def static_mode():
    paddle.enable_static()
    yield
    paddle.disable_static()


def test_shape_tensor_drives_reshape_at_run_time(static_mode):
    main, st = paddle.static.Program(), paddle.static.Program()
    with paddle.static.program_guard(main, st):
        x = paddle.static.data('x', [None, 6], 'float32')
        s = paddle.shape(x)
        y = paddle.reshape(x, [s[0], 3, 2])
        z = paddle.reshape(y * 2, [s[0], -1])
        w = paddle.reshape(x, s)
    assert y.shape == [-1, 3, 2] and z.shape == [-1, 6] and w.shape == [-1, 6] and s.shape == [2]
    exe = paddle.static.Executor(paddle.CPUPlace())
    for B in (5, 9):
        xs = np.arange(B * 6, dtype='float32').reshape(B, 6)
        a, b, c, d = exe.run(main, feed={'x': xs}, fetch_list=[s, y, z, w])
        assert a.tolist() == [B, 6]
        assert b.shape == (B, 3, 2) and c.shape == (B, 6) and d.shape == (B, 6)
        np.testing.assert_allclose(c, xs * 2)
        np.testing.assert_allclose(b.reshape(B, 6), xs)
