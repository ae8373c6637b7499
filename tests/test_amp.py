"""AMP semantics vs the reference (python/paddle/amp/auto_cast.py:383, amp_lists.py, debugging.py)."""
import os

import numpy as np
import pytest

import paddle
import paddle.nn.functional as F


def _x(*shape):
    return paddle.to_tensor(np.random.RandomState(0).randn(*shape).astype('float32'))


def test_o1_white_black_lists():
    lin = paddle.nn.Linear(8, 8)
    x = _x(4, 8)
    with paddle.amp.auto_cast(level='O1', dtype='bfloat16'):
        y = lin(x)
        assert y.dtype == paddle.bfloat16           # matmul_v2: white
        s = F.softmax(y)
        assert s.dtype == paddle.float32            # softmax: black in O1
        ln = F.layer_norm(y, [8])
        assert ln.dtype == paddle.float32           # layer_norm: black
        z = paddle.exp(y)
        assert z.dtype == paddle.float32            # exp: black
        r = F.relu(y)
        assert r.dtype == paddle.bfloat16           # gray: follows its input
    y2 = lin(x)
    assert y2.dtype == paddle.float32               # outside the guard: untouched


def test_custom_lists_and_overlap():
    lin = paddle.nn.Linear(8, 8)
    x = _x(4, 8)
    with paddle.amp.auto_cast(custom_black_list=['matmul_v2'], dtype='bfloat16'):
        assert lin(x).dtype == paddle.float32
    with paddle.amp.auto_cast(custom_white_list=['softmax'], dtype='bfloat16'):
        assert F.softmax(x).dtype == paddle.bfloat16
    with pytest.raises(ValueError):
        with paddle.amp.auto_cast(custom_white_list=['softmax'], custom_black_list=['softmax']):
            pass
    with pytest.raises(ValueError):
        with paddle.amp.auto_cast(level='O3'):
            pass
    with pytest.raises(ValueError):
        with paddle.amp.auto_cast(dtype='float64'):
            pass


def test_o2_and_od_levels():
    x = _x(4, 8).astype('bfloat16')
    with paddle.amp.auto_cast(level='O2', dtype='bfloat16'):
        assert F.softmax(x).dtype == paddle.bfloat16      # pure low precision
        emb = paddle.nn.Embedding(10, 8)
        ids = paddle.to_tensor([[1, 2]])
        assert emb(ids).dtype == paddle.float32           # lookup_table_v2: extra black list
    with paddle.amp.auto_cast(level='OD', dtype='bfloat16'):
        assert F.softmax(_x(2, 3)).dtype == paddle.float32  # OD: black list empty, softmax untouched
        assert paddle.matmul(_x(2, 3), _x(3, 2)).dtype == paddle.bfloat16
    with paddle.amp.auto_cast(enable=False, dtype='bfloat16'):
        assert paddle.matmul(_x(2, 3), _x(3, 2)).dtype == paddle.float32


def test_o1_grads_flow_to_fp32_params():
    lin = paddle.nn.Linear(8, 4)
    with paddle.amp.auto_cast(dtype='bfloat16'):
        loss = lin(_x(3, 8)).astype('float32').sum()
    loss.backward()
    assert lin.weight.grad is not None and lin.weight.grad.dtype == paddle.float32


def test_decorate_master_grad_and_save_dtype():
    model = paddle.nn.Sequential(paddle.nn.Linear(8, 8), paddle.nn.LayerNorm(8))
    opt = paddle.optimizer.AdamW(parameters=model.parameters())
    model, opt = paddle.amp.decorate(model, opt, level='O2', dtype='bfloat16', master_grad=True, save_dtype='float32')
    assert model[0].weight.dtype == paddle.bfloat16
    assert model[1].weight.dtype == paddle.float32       # norm layers stay fp32
    out = model(_x(2, 8).astype('bfloat16'))
    out.astype('float32').sum().backward()
    assert model[0].weight.grad.dtype == paddle.float32  # master_grad
    sd = model.state_dict()
    assert all(v.dtype == paddle.float32 for v in sd.values())
    opt.step()


def test_decorate_excluded_layers():
    model = paddle.nn.Sequential(paddle.nn.Linear(4, 4), paddle.nn.Linear(4, 4))
    model = paddle.amp.decorate(model, level='O2', dtype='bfloat16', excluded_layers=[model[1]])
    assert model[0].weight.dtype == paddle.bfloat16
    assert model[1].weight.dtype == paddle.float32


def test_operator_stats():
    from paddle.amp import debugging
    lin = paddle.nn.Linear(8, 8)
    debugging.enable_operator_stats_collection()
    with paddle.amp.auto_cast(dtype='bfloat16'):
        y = lin(_x(2, 8))
        F.softmax(y)
    table = debugging.disable_operator_stats_collection()
    assert table['matmul_v2'][1] == 1                    # one bf16 call
    assert table['softmax'][2] == 1                      # one fp32 call
    with debugging.collect_operator_stats():
        paddle.matmul(_x(2, 2), _x(2, 2))


def test_tensor_dump_and_compare_accuracy(tmp_path):
    from paddle.amp import debugging
    lin = paddle.nn.Linear(8, 8)
    x = _x(4, 8)
    d32, d16 = str(tmp_path / 'fp32'), str(tmp_path / 'bf16')
    cfg = debugging.TensorCheckerConfig(True, debugging.DebugMode.DUMP_ALL, output_dir=d32)
    debugging.enable_tensor_checker(cfg)
    F.softmax(lin(x))
    debugging.disable_tensor_checker()
    cfg = debugging.TensorCheckerConfig(True, debugging.DebugMode.DUMP_ALL, output_dir=d16)
    debugging.enable_tensor_checker(cfg)
    with paddle.amp.auto_cast(dtype='bfloat16'):
        F.softmax(lin(x))
    debugging.disable_tensor_checker()
    out = str(tmp_path / 'cmp.xlsx')
    bad = debugging.compare_accuracy(d32, d16, out, dump_all_tensors=True)
    rows = open(str(tmp_path / 'cmp.csv')).read().strip().split('\n')
    assert rows[0].startswith('tensor,') and len(rows) == 3  # header + matmul_v2 + softmax
    assert 'bfloat16' in rows[1] and bad == 0


def test_check_numerics_abort():
    from paddle.amp import debugging
    t = paddle.to_tensor([1.0, float('nan')])
    with pytest.raises(RuntimeError):
        debugging.check_numerics(t, 'op', 'x')
    stats, vals = debugging.check_numerics(t, 'op', 'x', debugging.DebugMode.CHECK_NAN_INF)
    assert stats.numpy().tolist()[:2] == [1, 0]


def test_matmul_operator_follows_amp_lists():
    """`a @ b` is matmul_v2 (white list): low precision under O1, and a bf16 activation times an fp32
    weight is cast instead of raising a dtype mismatch."""
    a, w = _x(4, 8), _x(8, 3)
    with paddle.amp.auto_cast(level='O1', dtype='bfloat16'):
        y = a @ w
        assert y.dtype == paddle.bfloat16
        h = paddle.nn.Linear(8, 8)(a)                # bf16 activation
        z = h @ w                                    # fp32 weight
        assert z.dtype == paddle.bfloat16
        r = w.t() @ a.t()                            # __matmul__ on the other operand order
        assert r.dtype == paddle.bfloat16
    y32 = a @ w
    assert y32.dtype == paddle.float32
    np.testing.assert_allclose(y.astype('float32').numpy(), y32.numpy(), rtol=3e-2, atol=3e-2)
