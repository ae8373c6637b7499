"""paddle.incubate (reference: python/paddle/incubate/__init__.py)."""
import torch

from . import nn  # noqa: F401
from . import autotune  # noqa: F401
from . import asp  # noqa: F401
from . import autograd  # noqa: F401
from .optimizer import LookAhead, ModelAverage  # noqa: F401
from . import optimizer  # noqa: F401
from ..core.tensor import _wrap, _unwrap
from ..geometric import (segment_sum, segment_mean, segment_max, segment_min,  # noqa: F401
                         send_u_recv as graph_send_recv, reindex_graph as graph_reindex,
                         sample_neighbors as graph_sample_neighbors)
from .. import ops as _ops


def softmax_mask_fuse_upper_triangle(x):
    """softmax(x + causal mask) over the last dim (reference fused_softmax_mask_upper_triangle)."""
    t = _unwrap(x)
    if _ops.use_hip(t):
        return _wrap(_ops.softmax.softmax_mask_upper_triangle(t))
    S = t.shape[-1]
    m = torch.ones(t.shape[-2], S, dtype=torch.bool, device=t.device).triu(1 + S - t.shape[-2])
    return _wrap(torch.softmax(t.float().masked_fill(m, float('-inf')), -1).to(t.dtype))


def softmax_mask_fuse(x, mask, name=None):
    t, m = _unwrap(x), _unwrap(mask)
    return _wrap(torch.softmax((t.float() + m.float()), -1).to(t.dtype))


def graph_khop_sampler(row, colptr, input_nodes, sample_sizes, sorted_eids=None, return_eids=False, name=None):
    """Multi-hop neighbour sampling: one sample_neighbors per hop, frontier = new nodes."""
    from ..geometric import sample_neighbors, reindex_graph
    nodes = input_nodes
    all_src, all_dst = [], []
    frontier = nodes
    for k in sample_sizes:
        nb, cnt = sample_neighbors(row, colptr, frontier, k)
        all_src.append(_unwrap(nb))
        all_dst.append(torch.repeat_interleave(_unwrap(frontier), _unwrap(cnt).long()))
        frontier = _wrap(torch.unique(_unwrap(nb)))
    src = torch.cat(all_src)
    dst = torch.cat(all_dst)
    s, d, out_nodes = reindex_graph(nodes, _wrap(src), _wrap(torch.bincount(
        torch.searchsorted(torch.unique(dst), dst), minlength=0)))
    return _wrap(src), _wrap(dst), out_nodes, None


def identity_loss(x, reduction="none"):
    t = _unwrap(x)
    if reduction in ('sum', 0):
        return _wrap(t.sum())
    if reduction in ('mean', 1):
        return _wrap(t.mean())
    return x


__all__ = ['LookAhead', 'ModelAverage', 'softmax_mask_fuse_upper_triangle', 'softmax_mask_fuse', 'graph_send_recv',
           'graph_khop_sampler', 'graph_sample_neighbors', 'graph_reindex', 'segment_sum', 'segment_mean',
           'segment_max', 'segment_min', 'identity_loss']


def __getattr__(name):
    if name == 'distributed':  # lazy: pulls in paddle.distributed
        import importlib
        m = importlib.import_module('.distributed', __name__)
        globals()[name] = m
        return m
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")
