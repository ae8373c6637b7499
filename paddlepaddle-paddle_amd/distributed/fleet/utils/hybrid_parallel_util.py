"""Hybrid-parallel helpers (reference: python/paddle/distributed/fleet/utils/hybrid_parallel_util.py)."""
import torch
import torch.distributed as dist

from ....core.tensor import _unwrap


def fused_allreduce_gradients(parameter_list, hcg):
    group = hcg.get_data_parallel_group() if hcg is not None else None
    if group is not None and group.nranks == 1:
        return
    grads = [p._t.grad for p in parameter_list if p._t.grad is not None]
    if not grads:
        return
    by_dt = {}
    for g in grads:
        by_dt.setdefault(g.dtype, []).append(g)
    for gs in by_dt.values():
        flat = torch.cat([g.reshape(-1) for g in gs])
        dist.all_reduce(flat, group=None if group is None else group.pg)
        flat.div_(group.nranks if group is not None else dist.get_world_size())
        off = 0
        for g in gs:
            n = g.numel()
            g.copy_(flat[off:off + n].view(g.shape))
            off += n


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
