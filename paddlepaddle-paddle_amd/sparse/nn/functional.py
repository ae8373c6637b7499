"""paddle.sparse.nn.functional (reference: python/paddle/sparse/nn/functional/{conv,pooling,
activation,transformer}.py; kernels paddle/phi/kernels/sparse/gpu/conv_kernel.cu).

Sparse convolution on COO voxel tensors [N, (D,) H, W, C] (sparse_dim = spatial rank + 1):
a *rulebook* lists, per kernel offset, the (input row, output row) pairs that meet; each offset
is then one dense GEMM of the gathered input rows with that offset's [Cin, Cout] weight slice
(hipBLASLt), scatter-added into the output rows.  Coordinates are matched by sorted int64 keys
(``searchsorted``) on the device — no host hashing.
"""
import itertools

import torch

from ...core.tensor import _wrap, _unwrap


def _tuple(v, n):
    return (v,) * n if isinstance(v, int) else tuple(v)


def _keys(coords, dims):
    """coords [nsd, nnz] (batch + spatial) → int64 keys."""
    k = coords[0].clone()
    for i, d in enumerate(dims):
        k = k * d + coords[i + 1]
    return k


def _rulebook(coords, spatial, ksize, stride, padding, dilation, subm):
    """Returns (out_coords [nsd, n_out], out_spatial, [(k_index, in_idx, out_idx), ...])."""
    nd = len(spatial)
    dev = coords.device
    if subm:
        out_spatial = spatial
    else:
        out_spatial = tuple((spatial[i] + 2 * padding[i] - dilation[i] * (ksize[i] - 1) - 1) // stride[i] + 1
                            for i in range(nd))
    offsets = list(itertools.product(*[range(k) for k in ksize]))
    if subm:
        out_coords = coords
        keys = _keys(coords, spatial)
        order = torch.argsort(keys)
        skeys = keys[order]
        rules = []
        center = tuple((k - 1) // 2 for k in ksize)
        for ki, off in enumerate(offsets):
            # input = output + (off - center) * dilation
            cand = coords.clone()
            valid = torch.ones(coords.shape[1], dtype=torch.bool, device=dev)
            for d in range(nd):
                cand[d + 1] = coords[d + 1] + (off[d] - center[d]) * dilation[d]
                valid &= (cand[d + 1] >= 0) & (cand[d + 1] < spatial[d])
            ck = _keys(cand, spatial)
            pos = torch.searchsorted(skeys, ck).clamp(max=max(skeys.numel() - 1, 0))
            hit = valid & (skeys[pos] == ck) if skeys.numel() else valid & False
            out_idx = torch.nonzero(hit).squeeze(1)
            in_idx = order[pos[hit]]
            if out_idx.numel():
                rules.append((ki, in_idx, out_idx))
        return out_coords, out_spatial, rules
    # regular conv: every (input, offset) that lands on a stride-aligned output
    cands, kidx, iidx = [], [], []
    for ki, off in enumerate(offsets):
        oc = coords.clone()
        valid = torch.ones(coords.shape[1], dtype=torch.bool, device=dev)
        for d in range(nd):
            num = coords[d + 1] + padding[d] - off[d] * dilation[d]
            valid &= (num >= 0) & (num % stride[d] == 0)
            o = torch.div(num, stride[d], rounding_mode='floor')
            valid &= o < out_spatial[d]
            oc[d + 1] = o
        sel = torch.nonzero(valid).squeeze(1)
        cands.append(oc[:, sel])
        kidx.append(torch.full((sel.numel(),), ki, device=dev, dtype=torch.long))
        iidx.append(sel)
    allc = torch.cat(cands, 1)
    allk = torch.cat(kidx)
    alli = torch.cat(iidx)
    keys = _keys(allc, out_spatial)
    uniq, inv = torch.unique(keys, return_inverse=True)
    # decode unique keys back to coordinates
    out_coords = torch.empty(coords.shape[0], uniq.numel(), dtype=coords.dtype, device=dev)
    rem = uniq.clone()
    for d in range(nd - 1, -1, -1):
        out_coords[d + 1] = rem % out_spatial[d]
        rem = torch.div(rem, out_spatial[d], rounding_mode='floor')
    out_coords[0] = rem
    rules = []
    for ki in range(len(offsets)):
        m = allk == ki
        if m.any():
            rules.append((ki, alli[m], inv[m]))
    return out_coords, out_spatial, rules


def _conv(x, weight, bias, stride, padding, dilation, groups, subm, nd, data_format):
    t = _unwrap(x).coalesce()
    w = _unwrap(weight)                           # [k..., Cin/groups, Cout]
    coords, feats = t.indices(), t.values()       # [nd+1, nnz], [nnz, Cin]
    spatial = tuple(t.shape[1:1 + nd])
    ksize = tuple(w.shape[:nd])
    stride, padding, dilation = _tuple(stride, nd), _tuple(padding, nd), _tuple(dilation, nd)
    out_coords, out_spatial, rules = _rulebook(coords, spatial, ksize, stride, padding, dilation, subm)
    cout = w.shape[-1]
    wk = w.reshape(-1, w.shape[-2], cout)
    out = torch.zeros(out_coords.shape[1], cout, dtype=feats.dtype, device=feats.device)
    if groups == 1:
        for ki, ii, oi in rules:
            out.index_add_(0, oi, feats.index_select(0, ii) @ wk[ki])
    else:
        cin_g, cout_g = w.shape[-2], cout // groups
        for ki, ii, oi in rules:
            f = feats.index_select(0, ii)
            parts = [f[:, g * cin_g:(g + 1) * cin_g] @ wk[ki][:, g * cout_g:(g + 1) * cout_g] for g in range(groups)]
            out.index_add_(0, oi, torch.cat(parts, 1))
    if bias is not None:
        out = out + _unwrap(bias)
    shape = (t.shape[0],) + tuple(out_spatial) + (cout,)
    return _wrap(torch.sparse_coo_tensor(out_coords, out, shape).coalesce())


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NHWC", name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, False, 2, data_format)


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, False, 3, data_format)


def subm_conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NHWC", key=None,
                name=None):
    return _conv(x, weight, bias, 1, padding, dilation, groups, True, 2, data_format)


def subm_conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", key=None,
                name=None):
    return _conv(x, weight, bias, 1, padding, dilation, groups, True, 3, data_format)


subm_conv2d_igemm = subm_conv2d
subm_conv3d_igemm = subm_conv3d


def max_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NDHWC", name=None):
    t = _unwrap(x).coalesce()
    coords, feats = t.indices(), t.values()
    ks = _tuple(kernel_size, 3)
    st = _tuple(stride if stride is not None else kernel_size, 3)
    pd = _tuple(padding, 3)
    out_coords, out_spatial, rules = _rulebook(coords, tuple(t.shape[1:4]), ks, st, pd, (1, 1, 1), False)
    out = torch.full((out_coords.shape[1], feats.shape[1]), float('-inf'), dtype=feats.dtype, device=feats.device)
    for _, ii, oi in rules:
        out = out.index_reduce(0, oi, feats.index_select(0, ii), 'amax', include_self=True)
    shape = (t.shape[0],) + tuple(out_spatial) + (feats.shape[1],)
    return _wrap(torch.sparse_coo_tensor(out_coords, out, shape).coalesce())


def _values_act(fn):
    def op(x, *a, name=None, **k):
        from .. import _map_values
        return _map_values(x, lambda v: fn(v, *a, **k))
    return op


relu = _values_act(torch.relu)
relu6 = _values_act(lambda v: torch.clamp(v, 0, 6))
leaky_relu = _values_act(lambda v, negative_slope=0.01: torch.nn.functional.leaky_relu(v, negative_slope))


def softmax(x, axis=-1, name=None):
    """Row softmax over the stored entries of a CSR (or COO) matrix; zeros stay implicit."""
    t = _unwrap(x)
    csr = t.layout == torch.sparse_csr
    c = t.to_sparse_coo().coalesce() if csr else t.coalesce()
    out = torch.sparse.softmax(c, dim=axis if axis >= 0 else c.dim() + axis).coalesce()
    return _wrap(out.to_sparse_csr() if csr else out)


def attention(query, key, value, sparse_mask, key_padding_mask=None, attn_mask=None, name=None):
    """softmax(QK^T/sqrt(d) restricted to ``sparse_mask``'s nonzeros) @ V; q/k/v [B, H, S, D],
    sparse_mask CSR [B*H, S, S]."""
    q, k, v = _unwrap(query), _unwrap(key), _unwrap(value)
    B, H, S, D = q.shape
    m = _unwrap(sparse_mask).to_dense().reshape(B, H, S, S) != 0
    s = (q @ k.transpose(-1, -2)) / (D ** 0.5)
    if key_padding_mask is not None:
        m = m & (_unwrap(key_padding_mask).reshape(B, 1, 1, S) != 0)
    if attn_mask is not None:
        m = m & (_unwrap(attn_mask).reshape(1, 1, S, S) != 0)
    s = s.masked_fill(~m, float('-inf'))
    p = torch.softmax(s, -1).nan_to_num(0.0)
    return _wrap(p @ v)
