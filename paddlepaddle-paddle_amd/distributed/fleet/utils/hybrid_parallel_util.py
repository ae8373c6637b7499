"""Hybrid-parallel helpers (reference: python/paddle/distributed/fleet/utils/hybrid_parallel_util.py).

Gradient synchronisation over the data-parallel and segment-parallel (``sep``) axes follows the
reference's rule (hybrid_parallel_util.py:241-262): the reduction group is dp, sep, or the fused
dp x sep group; the sum is scaled by 1/dp only — sep ranks hold different sequence segments of
the SAME samples, so their partial gradients add up to the full gradient ("sep all reduce is not
scaled").

MI355X design: gradients that live in flat buffers (parallel/flat_buffer.py) are reduced in place
as contiguous slices of the flat gradient buffer, in buckets of ``bucket_size`` bytes, every
bucket's collective launched asynchronously before the first is waited for (RCCL rings over the
xGMI links then stream back to back); loose gradients are packed per bucket only.  Models wrapped
by ``TensorParallel`` / ``SegmentParallel`` reduce during backward instead (a hook-driven
``GradAllReducer`` on the dp x sep group), and these helpers skip the parameters it covers.
"""
import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 128 * 1024 * 1024


def dp_sep_group_and_scale(hcg):
    """(group, scale) of the gradient all-reduce over the data and sep axes (None when both are 1)."""
    if hcg is None:
        return None, None
    dp_on = hcg.get_data_parallel_world_size() > 1
    sep_on = hcg.get_sep_parallel_world_size() > 1
    if not (dp_on or sep_on):
        return None, None
    group, scale = None, 1.0
    if dp_on:
        group = hcg.get_data_parallel_group()
        scale = 1.0 / group.nranks
    if sep_on:
        group = hcg.get_sep_parallel_group() if group is None else hcg.get_dp_sep_parallel_group()
    return group, scale


def _pg(group):
    return None if group is None else getattr(group, 'pg', group)


def _buckets(grads, bucket_size):
    """Cut a list of gradients into runs of at most ``bucket_size`` bytes (one per dtype/device);
    a run of views that tile one flat buffer contiguously is reduced in place."""
    by_key = {}
    for g in grads:
        by_key.setdefault((g.dtype, g.device), []).append(g)
    out = []
    for gs in by_key.values():
        cur, nb = [], 0
        for g in gs:
            b = g.numel() * g.element_size()
            if cur and nb + b > bucket_size:
                out.append(cur)
                cur, nb = [], 0
            cur.append(g)
            nb += b
        if cur:
            out.append(cur)
    return out


def _contiguous_run(gs):
    """The single tensor that covers ``gs`` in place, if they are adjacent views of one storage."""
    if not all(g.is_contiguous() for g in gs):
        return None
    from ....parallel.flat_buffer import ALIGN
    st = gs[0].untyped_storage()
    es = gs[0].element_size()
    for g in gs[1:]:
        if g.untyped_storage().data_ptr() != st.data_ptr():
            return None
    # adjacent flat-buffer views are separated by at most their alignment padding (never by
    # another parameter's gradient, which could then be reduced twice): reduce the span
    for a, b in zip(gs[:-1], gs[1:]):
        gap = b.data_ptr() - (a.data_ptr() + a.numel() * es)
        if gap < 0 or gap >= ALIGN * es:
            return None
    lo = gs[0].data_ptr()
    span = (gs[-1].data_ptr() + gs[-1].numel() * es - lo) // es
    off = (lo - st.data_ptr()) // es
    return torch.empty(0, dtype=gs[0].dtype, device=gs[0].device).set_(st, off, (span,), (1,))


def fused_allreduce_gradients_with_group(parameter_list, group, bucket_size=DEFAULT_BUCKET_BYTES, scale=None):
    """All-reduce (sum, then ``scale``; default: average over the group) the gradients of
    ``parameter_list`` over ``group`` in buckets, every bucket in flight at once."""
    pg = _pg(group)
    if not dist.is_initialized():
        return
    world = dist.get_world_size(pg)
    if world == 1:
        return
    if scale is None:
        scale = 1.0 / world
    grads = [p._t.grad for p in parameter_list
             if p._t.grad is not None and p.__dict__.get('_hook_reduced') is None]
    if not grads:
        return
    works = []
    with torch.no_grad():
        for gs in _buckets(grads, bucket_size):
            run = _contiguous_run(gs)
            flat = run if run is not None else torch.cat([g.reshape(-1) for g in gs])
            works.append((gs, flat, run is not None, dist.all_reduce(flat, group=pg, async_op=True)))
        for gs, flat, inplace, w in works:
            w.wait()
            if scale != 1.0:
                flat.mul_(scale)
            if not inplace:
                off = 0
                for g in gs:
                    n = g.numel()
                    g.copy_(flat[off:off + n].view(g.shape))
                    off += n


def fused_allreduce_gradients(parameter_list, hcg):
    """Gradient sync over dp / sep / dp x sep (reference hybrid_parallel_util.py:241)."""
    if hcg is None:
        fused_allreduce_gradients_with_group(parameter_list, None)
        return
    group, scale = dp_sep_group_and_scale(hcg)
    if group is None:
        return
    fused_allreduce_gradients_with_group(parameter_list, group, scale=scale)


def _broadcast(model, group, src):
    if group is None or group.nranks == 1:
        return
    with torch.no_grad():
        for p in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(p._t, src, group=group.pg)


def broadcast_mp_parameters(model, hcg):
    _broadcast(model, hcg.get_model_parallel_group(), hcg.get_model_parallel_group_src_rank())


def broadcast_dp_parameters(model, hcg):
    _broadcast(model, hcg.get_data_parallel_group(), hcg.get_data_parallel_group_src_rank())


def broadcast_sharding_parameters(model, hcg):
    _broadcast(model, hcg.get_sharding_parallel_group(), hcg.get_sharding_parallel_group_src_rank())


def broadcast_sep_parameters(model, hcg):
    """reference hybrid_parallel_util.py:275: every sep rank starts from the same weights."""
    _broadcast(model, hcg.get_sep_parallel_group(), hcg.get_sep_parallel_group_src_rank())


def install_grad_sync(model, hcg, bucket_mb=64):
    """Overlap the dp / sep gradient all-reduce with backward: a hook-driven bucketed reducer on
    the dp x sep group (scaled by 1/dp) over every trainable parameter of ``model``, tensor-parallel
    shards included.  Returns the reducer (None when neither axis is > 1)."""
    group, scale = dp_sep_group_and_scale(hcg)
    if group is None or not dist.is_initialized():
        return None
    from ....parallel.data_parallel import GradAllReducer
    return GradAllReducer(model.parameters(), group, max(int(bucket_mb), 1), average=False, scale=scale,
                          include_distributed=True)
