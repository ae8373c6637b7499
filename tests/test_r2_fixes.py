"""Regression tests for round-2 correctness fixes (CPU): cross_entropy axis shapes, the reference
paddle.save/.pdparams layout (plain ndarrays + name table, big-parameter slices), GQA packed
flash attention, paddle.distributed.io."""
import io
import pickle

import numpy as np
import pytest
import torch

import paddle
import paddle.nn.functional as F


@pytest.mark.parametrize("axis", [0, 1, 2, -1])
def test_cross_entropy_none_keeps_label_shape(axis):
    paddle.seed(0)
    x = paddle.randn([2, 3, 4])
    shape = [2, 3, 4]
    shape[axis] = 1
    n = x.shape[axis]
    lab = paddle.randint(0, n, shape)
    out = F.cross_entropy(x, lab, reduction='none', axis=axis)
    assert list(out.shape) == shape  # reference: label-shaped, unit dim at `axis`
    # value check against log_softmax along the axis
    lp = torch.log_softmax(x._t.float(), axis)
    want = -torch.gather(lp, axis % 3, lab._t.long())
    np.testing.assert_allclose(out.numpy(), want.numpy(), rtol=1e-5, atol=1e-6)
    mean = F.cross_entropy(x, lab, reduction='mean', axis=axis)
    np.testing.assert_allclose(float(mean), float(want.mean()), rtol=1e-5)


def test_softmax_with_cross_entropy_axis():
    x = paddle.randn([4, 5, 6])
    lab = paddle.randint(0, 5, [4, 1, 6])
    out = F.softmax_with_cross_entropy(x, lab, axis=1)
    assert list(out.shape) == [4, 1, 6]


def _raw_pickle(path):
    with open(path, 'rb') as f:
        return pickle.loads(f.read())  # our own file (test fixture), not reference-shipped data


def test_state_dict_saved_as_plain_ndarrays(tmp_path):
    lin = paddle.nn.Linear(3, 4)
    p = str(tmp_path / 'm.pdparams')
    paddle.save(lin.state_dict(), p)
    raw = _raw_pickle(p)
    assert isinstance(raw['weight'], np.ndarray) and raw['weight'].shape == (3, 4)
    assert raw['StructuredToParameterName@@'] == {'weight': lin.weight.name, 'bias': lin.bias.name}
    back = paddle.load(p)
    assert 'StructuredToParameterName@@' not in back
    assert back['weight'].name == lin.weight.name
    np.testing.assert_array_equal(back['weight'].numpy(), lin.weight.numpy())
    keep = paddle.load(p, keep_name_table=True)
    assert 'StructuredToParameterName@@' in keep
    npy = paddle.load(p, return_numpy=True)
    assert isinstance(npy['bias'], np.ndarray)


def test_bf16_state_dict_uint16_roundtrip(tmp_path):
    t = paddle.to_tensor(torch.randn(5, 7).bfloat16())
    p = str(tmp_path / 'b.pdparams')
    paddle.save({'w': t}, p)
    raw = _raw_pickle(p)
    assert raw['w'].dtype == np.uint16
    back = paddle.load(p)
    assert back['w']._t.dtype == torch.bfloat16
    assert torch.equal(back['w']._t, t._t)


def test_nested_object_uses_name_tuples(tmp_path):
    lin = paddle.nn.Linear(2, 2)
    obj = {'model': lin.state_dict(), 'epoch': 3, 'lst': [lin.weight]}
    p = str(tmp_path / 'ck.pd')
    paddle.save(obj, p)
    raw = _raw_pickle(p)
    assert isinstance(raw['lst'][0], tuple) and raw['lst'][0][0] == lin.weight.name
    back = paddle.load(p)
    assert back['epoch'] == 3
    assert back['lst'][0].name == lin.weight.name
    np.testing.assert_array_equal(back['model']['bias'].numpy(), lin.bias.numpy())


def test_big_param_slices_reassembled():
    """A protocol-2 file whose parameter was split into UnpackBigParamInfor@@ slices (the
    reference's >1 GB path, io_utils.py:236) loads as one reassembled parameter."""
    full = np.arange(24, dtype=np.float32).reshape(4, 6)
    flat = full.reshape(-1)
    obj = {'w@@.0': flat[:10], 'w@@.1': flat[10:20], 'w@@.2': flat[20:],
           'b': np.ones(3, np.float32),
           'UnpackBigParamInfor@@': {'w': {'OriginShape': (4, 6), 'slices': ['w@@.0', 'w@@.1', 'w@@.2']}},
           'StructuredToParameterName@@': {'w': 'linear_0.w_0', 'b': 'linear_0.b_0'}}
    buf = io.BytesIO(pickle.dumps(obj, protocol=2))
    back = paddle.load(buf)
    assert set(back.keys()) == {'w', 'b'}
    np.testing.assert_array_equal(back['w'].numpy(), full)
    assert back['w'].name == 'linear_0.w_0'


def test_unpack_saved_dict_splits_big_arrays():
    from paddle.framework import io as pio
    x = np.arange(50, dtype=np.float32).reshape(5, 10)
    saved = pio._unpack_saved_dict({'x': x.copy(), 'y': np.ones(2, np.float32)}, 2, max_bytes=81)  # 20 elems/slice
    assert saved['UnpackBigParamInfor@@']['x']['slices'] == ['x@@.0', 'x@@.1', 'x@@.2']
    assert 'x' not in saved and saved['x@@.2'].shape == (10,)
    back = pio._pack_loaded_dict(saved)
    np.testing.assert_array_equal(back['x'], x)
    assert pio._unpack_saved_dict({'x': x.copy()}, 4, max_bytes=81).keys() == {'x'}  # protocol 4: no split


def test_restricted_unpickler_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (eval, ("1+1",))
    p = tmp_path / 'evil.pd'
    p.write_bytes(pickle.dumps({'x': Evil()}))
    with pytest.raises(ValueError):
        paddle.load(str(p))


def test_qkvpacked_gqa_slicing():
    """[b, s, hq/hk + 2, hk, d] packing: query groups first, then k, then v (reference
    flash_attention.py:425); compared with the unpacked call."""
    torch.manual_seed(0)
    b, s, hk, g, d = 2, 8, 2, 3, 16
    t = torch.randn(b, s, g + 2, hk, d)
    out = F.flash_attn_qkvpacked(paddle.to_tensor(t), causal=True)[0]
    q = t[:, :, :-2].reshape(b, s, g * hk, d)
    ref = F.flash_attention(paddle.to_tensor(q), paddle.to_tensor(t[:, :, -2]), paddle.to_tensor(t[:, :, -1]),
                            causal=True)[0]
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    assert list(out.shape) == [b, s, g * hk, d]


def test_distributed_io_importable():
    import paddle.distributed.io as dio
    assert callable(dio.save_persistables) and callable(dio.load_persistables)
    assert callable(dio.load_inference_model_distributed) and callable(dio.is_persistable)


def test_distributed_io_persistables_roundtrip(tmp_path):
    import paddle.distributed.io as dio
    from paddle.static import proto
    paddle.enable_static()
    try:
        main, start = paddle.static.Program(), paddle.static.Program()
        with paddle.static.program_guard(main, start):
            x = paddle.static.data('x', [None, 4], 'float32')
            y = paddle.static.nn.fc(x, 3)
        params = main.all_parameters()
        assert params and all(dio.is_persistable(p) for p in params)
        dio.save_persistables(None, str(tmp_path / 'sep'), main)
        dio.save_persistables(None, str(tmp_path / 'comb'), main, filename='all.pdiparams')
        saved = {p.name: p._t.clone() for p in params}
        # each per-variable file is one reference LoDTensor stream
        with open(tmp_path / 'sep' / params[0].name, 'rb') as f:
            t, lod = proto.tensor_from_stream(f)
        assert torch.equal(t, saved[params[0].name]) and lod == []
        for p in params:
            p._t.data.zero_()
        dio.load_persistables(None, str(tmp_path / 'comb'), main, filename='all.pdiparams')
        for p in params:
            assert torch.equal(p._t, saved[p.name])
        for p in params:
            p._t.data.zero_()
        dio.load_persistables(None, str(tmp_path / 'sep'), main)
        for p in params:
            assert torch.equal(p._t, saved[p.name])
    finally:
        paddle.disable_static()


def test_lod_tensor_stream_layout():
    """Byte layout of one LoDTensor stream (reference lod_tensor.cc:205 / tensor_util.cc:455)."""
    import struct
    from paddle.static import proto
    t = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    b = proto.tensor_to_stream(t, lod=[[0, 1, 2]])
    assert struct.unpack('<I', b[:4])[0] == 0
    assert struct.unpack('<Q', b[4:12])[0] == 1            # one LoD level
    assert struct.unpack('<Q', b[12:20])[0] == 24           # 3 x uint64 offsets
    off = 20 + 24
    assert struct.unpack('<I', b[off:off + 4])[0] == 0
    dsz = struct.unpack('<i', b[off + 4:off + 8])[0]
    desc = proto.VarType.TensorDesc()
    desc.ParseFromString(b[off + 8:off + 8 + dsz])
    assert desc.data_type == 5 and list(desc.dims) == [2, 3]
    assert b[off + 8 + dsz:] == t.numpy().tobytes()
    back, lod = proto.tensor_from_stream(io.BytesIO(b))
    assert torch.equal(back, t) and lod == [[0, 1, 2]]
