"""paddle.geometric (reference: python/paddle/geometric/ — math.py segment_*, message_passing/
send_recv.py send_u_recv:36 / send_ue_recv:187 / send_uv:392, reindex.py, sampling/neighbors.py).

Message passing = gather rows by ``src_index`` + scatter-reduce into ``dst_index`` rows
(``index_reduce``/``index_add`` device kernels); rows receiving nothing are 0 for every reduce
op, as in the reference.
"""
import warnings

import torch

from .core.tensor import _wrap, _unwrap

warnings.filterwarnings('ignore', message='index_reduce')


def _reduce_rows(msg, dst, n, op):
    dst = dst.long()
    shape = (n,) + tuple(msg.shape[1:])
    if op == 'sum':
        return torch.zeros(shape, dtype=msg.dtype, device=msg.device).index_add_(0, dst, msg)
    if op == 'mean':
        s = torch.zeros(shape, dtype=msg.dtype, device=msg.device).index_add_(0, dst, msg)
        cnt = torch.zeros(n, dtype=msg.dtype, device=msg.device).index_add_(0, dst, torch.ones_like(dst, dtype=msg.dtype))
        return s / cnt.clamp(min=1).reshape((n,) + (1,) * (msg.dim() - 1))
    if op in ('max', 'min'):
        out = torch.zeros(shape, dtype=msg.dtype, device=msg.device)
        out = out.index_reduce(0, dst, msg, 'amax' if op == 'max' else 'amin', include_self=False)
        return out
    raise ValueError(f"reduce_op should be sum/mean/max/min, got {op}")


def _nseg(ids):
    return int(ids.max().item()) + 1 if ids.numel() else 0


def segment_sum(data, segment_ids, name=None):
    d, ids = _unwrap(data), _unwrap(segment_ids)
    return _wrap(_reduce_rows(d, ids, _nseg(ids), 'sum'))


def segment_mean(data, segment_ids, name=None):
    d, ids = _unwrap(data), _unwrap(segment_ids)
    return _wrap(_reduce_rows(d, ids, _nseg(ids), 'mean'))


def segment_min(data, segment_ids, name=None):
    d, ids = _unwrap(data), _unwrap(segment_ids)
    return _wrap(_reduce_rows(d, ids, _nseg(ids), 'min'))


def segment_max(data, segment_ids, name=None):
    d, ids = _unwrap(data), _unwrap(segment_ids)
    return _wrap(_reduce_rows(d, ids, _nseg(ids), 'max'))


def _out_n(x, out_size):
    if out_size is None:
        return x.shape[0]
    n = int(_unwrap(out_size).item()) if not isinstance(out_size, int) else out_size
    return n if n > 0 else x.shape[0]


def send_u_recv(x, src_index, dst_index, reduce_op="sum", out_size=None, name=None):
    t = _unwrap(x)
    msg = t.index_select(0, _unwrap(src_index).long())
    return _wrap(_reduce_rows(msg, _unwrap(dst_index), _out_n(t, out_size), reduce_op.lower()))


def _message(a, b, op):
    op = op.lower()
    if op == 'add':
        return a + b
    if op == 'sub':
        return a - b
    if op == 'mul':
        return a * b
    if op == 'div':
        return a / b
    raise ValueError(f"message_op should be add/sub/mul/div, got {op}")


def send_ue_recv(x, y, src_index, dst_index, message_op="add", reduce_op="sum", out_size=None, name=None):
    t, e = _unwrap(x), _unwrap(y)
    xs = t.index_select(0, _unwrap(src_index).long())
    while e.dim() < xs.dim():
        e = e.unsqueeze(-1)
    msg = _message(xs, e, message_op)
    return _wrap(_reduce_rows(msg, _unwrap(dst_index), _out_n(t, out_size), reduce_op.lower()))


def send_uv(x, y, src_index, dst_index, message_op="add", name=None):
    a = _unwrap(x).index_select(0, _unwrap(src_index).long())
    b = _unwrap(y).index_select(0, _unwrap(dst_index).long())
    return _wrap(_message(a, b, message_op))


def reindex_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    """Relabels ``x`` then first-seen new neighbours to 0..n-1; returns (src, dst, out_nodes)."""
    xs, nb, cnt = _unwrap(x), _unwrap(neighbors), _unwrap(count)
    dev = xs.device
    order = {}
    for v in xs.tolist():
        order.setdefault(v, len(order))
    for v in nb.tolist():
        order.setdefault(v, len(order))
    out_nodes = torch.tensor(list(order.keys()), dtype=xs.dtype, device=dev)
    src = torch.tensor([order[v] for v in nb.tolist()], dtype=xs.dtype, device=dev)
    dst = torch.repeat_interleave(torch.arange(xs.numel(), device=dev, dtype=xs.dtype), cnt.long())
    return _wrap(src), _wrap(dst), _wrap(out_nodes)


def reindex_heter_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    xs = _unwrap(x)
    nbs = [_unwrap(n) for n in neighbors]
    cnts = [_unwrap(c) for c in count]
    order = {}
    for v in xs.tolist():
        order.setdefault(v, len(order))
    srcs, dsts = [], []
    for nb, cnt in zip(nbs, cnts):
        for v in nb.tolist():
            order.setdefault(v, len(order))
        srcs.append(torch.tensor([order[v] for v in nb.tolist()], dtype=xs.dtype, device=xs.device))
        dsts.append(torch.repeat_interleave(torch.arange(xs.numel(), device=xs.device, dtype=xs.dtype), cnt.long()))
    out_nodes = torch.tensor(list(order.keys()), dtype=xs.dtype, device=xs.device)
    return _wrap(torch.cat(srcs)), _wrap(torch.cat(dsts)), _wrap(out_nodes)


def _sample(row, colptr, nodes, k, weights=None, eids=None, return_eids=False):
    r, cp, nd = _unwrap(row), _unwrap(colptr), _unwrap(nodes)
    out, cnts, oe = [], [], []
    w = _unwrap(weights) if weights is not None else None
    e = _unwrap(eids) if eids is not None else None
    for v in nd.tolist():
        lo, hi = int(cp[v]), int(cp[v + 1])
        deg = hi - lo
        if k < 0 or deg <= k:
            idx = torch.arange(lo, hi, device=r.device)
        elif w is None:
            idx = lo + torch.randperm(deg, device=r.device)[:k]
        else:
            idx = lo + torch.multinomial(w[lo:hi].float(), k, replacement=False)
        out.append(r[idx])
        cnts.append(idx.numel())
        if return_eids:
            oe.append(e[idx] if e is not None else idx)
    neighbors = torch.cat(out) if out else r[:0]
    count = torch.tensor(cnts, dtype=torch.int32, device=r.device)
    if return_eids:
        return _wrap(neighbors), _wrap(count), _wrap(torch.cat(oe) if oe else r[:0])
    return _wrap(neighbors), _wrap(count)


def sample_neighbors(row, colptr, input_nodes, sample_size=-1, eids=None, return_eids=False, perm_buffer=None,
                     name=None):
    return _sample(row, colptr, input_nodes, sample_size, None, eids, return_eids)


def weighted_sample_neighbors(row, colptr, edge_weight, input_nodes, sample_size=-1, eids=None, return_eids=False,
                              name=None):
    return _sample(row, colptr, input_nodes, sample_size, edge_weight, eids, return_eids)


__all__ = ['send_u_recv', 'send_ue_recv', 'send_uv', 'segment_sum', 'segment_mean', 'segment_min', 'segment_max',
           'reindex_graph', 'reindex_heter_graph', 'sample_neighbors', 'weighted_sample_neighbors']
