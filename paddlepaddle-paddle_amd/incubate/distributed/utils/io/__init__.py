"""Distributed save / load of dygraph state dicts.

Reference: python/paddle/incubate/distributed/utils/io/dist_save.py (save: gather the sharded
optimizer state of a sharding group to chosen ranks, then paddle.save), dist_load.py (load with
a target place), save_for_auto.py (per-rank parameters + a .pdattr file of dims mappings for
auto-parallel inference).  Gathers go through ``all_gather_object`` in groups of at most
``max_grouped_size`` bytes.
"""
import json
import os
import re

import torch

from .....core.tensor import Tensor, _wrap, _unwrap

__all__ = ['save', 'load', 'save_for_auto_inference']


def _dist():
    import torch.distributed as d
    return d if d.is_available() and d.is_initialized() else None


def _parse_size(s):
    if isinstance(s, int):
        return s
    m = re.fullmatch(r'([0-9]+)([GMK])', str(s))
    if not m:
        raise ValueError(f"Wrong max_size's format, the format must be like 10K, 9M, 200G, etc, or an integer. "
                         f"However this is {s}")
    return int(m.group(1)) * {'G': 1024 ** 3, 'M': 1024 ** 2, 'K': 1024}[m.group(2)]


def _nbytes(v):
    t = v._t if isinstance(v, Tensor) else v
    return t.numel() * t.element_size() if isinstance(t, torch.Tensor) else 64


def _cpu(v):
    if isinstance(v, Tensor):
        return v._t.detach().cpu()
    if isinstance(v, torch.Tensor):
        return v.detach().cpu()
    if isinstance(v, dict):
        return {k: _cpu(x) for k, x in v.items()}
    return v


def _groups(sd, max_size):
    cur, size = {}, 0
    for k, v in sd.items():
        b = _nbytes(v)
        if cur and size + b >= max_size:
            yield cur
            cur, size = {}, 0
        cur[k] = v
        size += b
    yield cur


def _sharding_group():
    try:
        from .....distributed import fleet
        hcg = fleet.get_hybrid_communicate_group()
    except Exception:
        return None, None
    if hcg is None:
        return None, None
    return hcg.get_sharding_parallel_group(), hcg


def _same_keys(sd, pg, d):
    keys = sorted(str(k) for k in sd)
    out = [None] * d.get_world_size(pg)
    d.all_gather_object(out, keys, group=pg)
    return all(o == keys for o in out)


def _gather_state_dict(sd, dst, group, d, max_size):
    pg = getattr(group, 'pg', group)
    n = d.get_world_size(pg)
    max_size = _parse_size(max_size) // max(n, 1)
    merged = {}
    local = list(_groups(sd, max_size))
    # every rank must join the same number of gathers
    counts = [None] * n
    d.all_gather_object(counts, len(local), group=pg)
    for i in range(max(counts)):
        piece = {k: _cpu(v) for k, v in local[i].items()} if i < len(local) else {}
        got = [None] * n
        d.all_gather_object(got, piece, group=pg)
        if d.get_rank() in dst:
            for g in got:
                for k, v in g.items():
                    merged.setdefault(k, v)
    if d.get_rank() in dst:
        return {k: (_wrap(v) if isinstance(v, torch.Tensor) else v) for k, v in merged.items()}
    return None


_SAVE_KEYS = ('protocol', 'use_binary_format', 'pickle_protocol')


def save(state_dict, path, **configs):
    """paddle.save of ``state_dict``; with ``gather_to`` and a sharding group of more than one rank,
    the optimizer state (``state_type='opt'``) of all sharding ranks is merged on the ``gather_to``
    ranks first."""
    import paddle
    kw = {k: v for k, v in configs.items() if k in _SAVE_KEYS}
    d = _dist()
    gather_to = configs.get('gather_to', None)
    if d is None or d.get_world_size() == 1 or gather_to is None:
        return paddle.save(state_dict, path, **kw)
    state_type = configs.get('state_type', None)
    if state_type not in ('params', 'opt'):
        raise AssertionError("must pass an arg state_type='params' or state_type='opt'")
    group, hcg = _sharding_group()
    if hcg is not None:
        assert hcg.get_model_parallel_world_size() == 1 and hcg.get_pipe_parallel_world_size() == 1, \
            "Only DP and Sharding is supported now."
    if state_type == 'params' or group is None or group.nranks == 1:
        return paddle.save(state_dict, path, **kw)
    pg = getattr(group, 'pg', group)
    if _same_keys(state_dict, pg, d):
        return paddle.save(state_dict, path, **kw)
    dst = [gather_to] if isinstance(gather_to, int) else list(gather_to)
    merged = _gather_state_dict(state_dict, dst, group, d, configs.get('max_grouped_size', '3G'))
    if d.get_rank() in dst:
        paddle.save(merged, path, **kw)


def load(path, **configs):
    """paddle.load; ``place`` ('cpu', 'gpu', 'gpu:N' or a Place) moves every tensor there."""
    import paddle
    place = configs.get('place', None)
    sd = paddle.load(path, **{k: v for k, v in configs.items() if k in ('return_numpy',)})
    if place is None:
        return sd
    s = str(place).lower()
    dev = torch.device('cpu') if 'cpu' in s else torch.device('cuda', int(s.split(':')[1]) if ':' in s else 0)

    def mv(v):
        if isinstance(v, Tensor):
            return _wrap(v._t.to(dev))
        if isinstance(v, dict):
            return {k: mv(x) for k, x in v.items()}
        return v
    return mv(sd)


def _dims_mapping(p):
    t = _unwrap(p)
    dm = [-1] * t.dim()
    if getattr(p, 'is_distributed', False):
        axis = getattr(p, 'split_axis', None)
        if axis is None:
            axis = 1 if t.dim() == 2 else 0
        dm[axis] = 1  # the model-parallel mesh axis
    return dm


def save_for_auto_inference(path_prefix, dist_model, cvt2cpu=False):
    """Writes ``{prefix}_dist{rank}.pdparams`` (the rank's full local parameters; a stage-3 model is
    gathered first) and ``{prefix}_dist{rank}.pdattr`` (JSON: process shape/group and dims mapping
    per parameter, mesh axes [dp*sharding, pp, mp])."""
    import paddle
    if path_prefix.endswith(os.sep):
        save_dir, base = path_prefix, 'saved_parameters'
    else:
        save_dir, base = os.path.dirname(path_prefix) or '.', os.path.basename(path_prefix)
    os.makedirs(save_dir, exist_ok=True)
    if hasattr(dist_model, 'get_all_parameters'):
        dist_model.get_all_parameters(cvt2cpu)
    sd = dist_model.state_dict()
    d = _dist()
    rank = d.get_rank() if d is not None else 0
    world = d.get_world_size() if d is not None else 1
    paddle.save(sd, os.path.join(save_dir, f"{base}_dist{rank}.pdparams"))
    _, hcg = _sharding_group() if world > 1 else (None, None)
    if hcg is not None:
        dp = hcg.get_data_parallel_world_size() * hcg.get_sharding_parallel_world_size()
        mp, pp = hcg.get_model_parallel_world_size(), hcg.get_pipe_parallel_world_size()
    else:
        dp, mp, pp = world, 1, 1
    attrs = {}
    for k, v in sd.items():
        if not isinstance(v, Tensor):
            continue
        attrs[k] = {'process_shape': [dp, pp, mp], 'process_group': list(range(world)),
                    'dims_mapping': _dims_mapping(v)}
    with open(os.path.join(save_dir, f"{base}_dist{rank}.pdattr"), 'w') as f:
        json.dump(attrs, f)
