"""paddle.sparse (COO/CSR, rulebook sparse conv vs dense conv) and paddle.geometric."""
import numpy as np
import torch

import paddle
import paddle.sparse as sp


def test_coo_csr_basics():
    idx = [[0, 1, 2], [1, 2, 0]]
    x = sp.sparse_coo_tensor(idx, [1.0, 2.0, 3.0], [3, 3])
    assert x.nnz() == 3 and x.is_sparse_coo()
    d = x.to_dense().numpy()
    assert d[0, 1] == 1 and d[2, 0] == 3
    y = sp.sin(x)
    np.testing.assert_allclose(y.values().numpy(), np.sin([1.0, 2.0, 3.0]), rtol=1e-6)
    csr = x.to_sparse_csr()
    assert csr.is_sparse_csr() and csr.crows().numpy().tolist() == [0, 1, 2, 3]
    dense = paddle.to_tensor(np.random.rand(3, 4).astype('float32'))
    np.testing.assert_allclose(sp.matmul(x, dense).numpy(), d @ dense.numpy(), rtol=1e-5)
    s = sp.add(x, x)
    np.testing.assert_allclose(s.to_dense().numpy(), 2 * d)
    a = paddle.to_tensor(np.random.rand(3, 5).astype('float32'))
    b = paddle.to_tensor(np.random.rand(5, 3).astype('float32'))
    mm = sp.masked_matmul(a, b, csr)
    ref = (a.numpy() @ b.numpy()) * (d != 0)
    np.testing.assert_allclose(mm.to_dense().numpy(), ref, rtol=1e-5)
    sm = sp.nn.functional.softmax(csr)
    assert abs(float(sm.to_dense().numpy().sum()) - 3.0) < 1e-5


def _dense_voxels(rng, N=1, D=5, H=6, W=7, C=3, p=0.3):
    occ = rng.rand(N, D, H, W) < p
    feats = rng.randn(N, D, H, W, C).astype('float32') * occ[..., None]
    return occ, feats


def test_subm_and_regular_sparse_conv3d_match_dense():
    rng = np.random.RandomState(0)
    occ, feats = _dense_voxels(rng)
    coords = np.stack(np.nonzero(occ))
    vals = feats[occ]
    x = sp.sparse_coo_tensor(coords, vals, list(feats.shape))
    w = rng.randn(3, 3, 3, 3, 4).astype('float32')
    wt = torch.from_numpy(w).permute(4, 3, 0, 1, 2)  # -> [Cout, Cin, kd, kh, kw]
    dense_in = torch.from_numpy(feats).permute(0, 4, 1, 2, 3)
    ref = torch.nn.functional.conv3d(dense_in, wt, padding=1).permute(0, 2, 3, 4, 1).numpy()
    out = sp.nn.functional.subm_conv3d(x, paddle.to_tensor(w), padding=1)
    got = out.to_dense().numpy()
    np.testing.assert_allclose(got[occ], ref[occ], rtol=1e-4, atol=1e-4)
    assert out.nnz() == occ.sum()
    out2 = sp.nn.functional.conv3d(x, paddle.to_tensor(w), stride=2, padding=1)
    ref2 = torch.nn.functional.conv3d(dense_in, wt, stride=2, padding=1).permute(0, 2, 3, 4, 1).numpy()
    np.testing.assert_allclose(out2.to_dense().numpy(), ref2, rtol=1e-4, atol=1e-4)
    layer = sp.nn.SubmConv3D(3, 8, 3, padding=1)
    bn = sp.nn.BatchNorm(8)
    y = sp.nn.ReLU()(bn(layer(x)))
    assert y.shape == [1, 5, 6, 7, 8]
    mp = sp.nn.functional.max_pool3d(x, 2, 2)
    assert mp.shape[1:4] == [2, 3, 3]


def test_geometric_ops():
    g = paddle.geometric
    x = paddle.to_tensor([[0., 2, 3], [1, 4, 5], [2, 6, 7]])
    src, dst = paddle.to_tensor([0, 1, 2, 0]), paddle.to_tensor([1, 2, 1, 0])
    assert g.send_u_recv(x, src, dst, 'sum').numpy().tolist() == [[0, 2, 3], [2, 8, 10], [1, 4, 5]]
    assert g.send_u_recv(x, src, dst, 'max').numpy().tolist() == [[0, 2, 3], [2, 6, 7], [1, 4, 5]]
    y = paddle.to_tensor([1., 1., 1., 1.])
    assert g.send_ue_recv(x, y, src, dst, 'add', 'sum').numpy().tolist() == [[1, 3, 4], [4, 10, 12], [2, 5, 6]]
    uv = g.send_uv(x, x, src, dst, 'mul')
    assert uv.shape == [4, 3]
    data = paddle.to_tensor([[1., 2], [3, 4], [5, 6]])
    ids = paddle.to_tensor([0, 0, 1])
    assert g.segment_sum(data, ids).numpy().tolist() == [[4, 6], [5, 6]]
    assert g.segment_mean(data, ids).numpy().tolist() == [[2, 3], [5, 6]]
    assert g.segment_min(data, ids).numpy().tolist() == [[1, 2], [5, 6]]
    row = paddle.to_tensor([3, 7, 0, 9, 1, 4, 2, 9, 3, 9, 1, 9, 7])
    colptr = paddle.to_tensor([0, 2, 4, 5, 6, 7, 9, 11, 11, 13, 13])
    nb, cnt = g.sample_neighbors(row, colptr, paddle.to_tensor([0, 8, 1, 2]), sample_size=2)
    assert cnt.numpy().tolist() == [2, 2, 2, 1]
