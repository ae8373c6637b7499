"""paddle dtypes are paddle DataType objects (reference: python/paddle/framework/dtype.py): they
print as ``paddle.float32``, equal and hash like the storage dtype, and are accepted everywhere a
dtype is taken."""
import os
import pickle
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import paddle  # noqa: E402


def test_prints_as_paddle_dtype():
    x = paddle.ones([2, 3])
    assert str(x.dtype) == 'paddle.float32' and repr(paddle.bfloat16) == 'paddle.bfloat16'
    assert isinstance(x.dtype, paddle.dtype)
    assert str(paddle.to_tensor([1, 2]).dtype) == 'paddle.int64'
    assert str(paddle.to_tensor([True]).dtype) == 'paddle.bool'


def test_equality_hash_and_attributes():
    x = paddle.ones([2], dtype='float16')
    assert x.dtype == paddle.float16 and x.dtype != paddle.float32
    assert x.dtype == torch.float16 and torch.float16 == x.dtype  # the storage dtype
    assert x.dtype in (paddle.float16, paddle.bfloat16)
    assert {paddle.float16: 'h'}[x.dtype] == 'h' and {torch.float16: 'h'}[x.dtype] == 'h'
    assert x.dtype.is_floating_point and paddle.float16.itemsize == 2
    assert not paddle.int32.is_floating_point
    assert x.dtype != 'float16'  # a DataType is not a string
    assert pickle.loads(pickle.dumps(paddle.bfloat16)) is paddle.bfloat16


def test_accepted_everywhere_a_dtype_is_taken():
    x = paddle.ones([3])
    for d in (paddle.float64, 'float64', np.float64, x.astype('float64').dtype):
        y = paddle.cast(x, d)
        assert y.dtype == paddle.float64
        assert paddle.zeros([2], dtype=d).dtype == paddle.float64
        assert paddle.to_tensor([1.0], dtype=d).dtype == paddle.float64
    assert x.astype(paddle.int32).dtype == paddle.int32
    assert paddle.finfo(paddle.bfloat16).bits == 16 and paddle.iinfo(paddle.int8).max == 127
    paddle.set_default_dtype(paddle.float64)
    try:
        assert paddle.get_default_dtype() == 'float64'
        assert paddle.nn.Linear(2, 2).weight.dtype == paddle.float64
    finally:
        paddle.set_default_dtype('float32')
    assert x.numpy().dtype == np.float32


def test_static_variables_and_input_spec_carry_paddle_dtypes():
    paddle.enable_static()
    try:
        main = paddle.static.Program()
        with paddle.static.program_guard(main):
            v = paddle.static.data('v', [-1, 4], paddle.bfloat16)
            assert v.dtype == paddle.bfloat16 and str(v.dtype) == 'paddle.bfloat16'
    finally:
        paddle.disable_static()
    spec = paddle.static.InputSpec([None, 4], paddle.float16, 'x')
    assert spec.dtype == paddle.float16 or str(spec.dtype).endswith('float16')
