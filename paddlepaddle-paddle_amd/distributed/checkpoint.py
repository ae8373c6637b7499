"""Distributed checkpoint (reference: python/paddle/distributed/checkpoint/save_state_dict.py,
load_state_dict.py, metadata.py).

Every rank writes only its own shards: ``<path>/<rank>_0.distcp`` (safetensors) holding each
local piece, and rank 0 writes ``<path>/0.metadata`` (JSON) mapping every global tensor to its
chunks (file, global offset, shape).  Loading works for any target layout: each rank computes
the global region its (possibly differently sharded) tensor covers and copies the overlapping
parts of every saved chunk — resharding on load, including a different world size.
Replicated tensors are written once (by the lowest rank holding them).
"""
import json
import os

import torch
import torch.distributed as dist

from ..core.tensor import Tensor, _unwrap


def _rank():
    return dist.get_rank() if dist.is_initialized() else 0


def _local_region(t):
    """(global_shape, offset) of this rank's piece; plain tensors are the whole tensor."""
    tt = _unwrap(t) if isinstance(t, Tensor) else t
    mesh = t.__dict__.get('process_mesh') if isinstance(t, Tensor) else None
    if mesh is None:
        return list(tt.shape), [0] * tt.dim(), True
    from .auto_parallel import Shard
    gshape = t.__dict__['_global_shape']
    off = [0] * len(gshape)
    c = mesh.coord(_rank())
    owner = True
    for d, p in enumerate(t.__dict__['placements']):
        if isinstance(p, Shard):
            n = mesh.shape[d]
            chunk = (gshape[p.dim] + n - 1) // n
            off[p.dim] += int(c[d]) * chunk
        elif c[d] != 0:
            owner = False  # replicated along this dim: only coordinate 0 writes
    return [int(v) for v in gshape], [int(v) for v in off], owner


def _flatten(sd, prefix=''):
    out = {}
    for k, v in sd.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            out.update(_flatten(v, key + '.'))
        else:
            out[key] = v
    return out


def save_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, async_save=False):
    from safetensors.torch import save_file
    os.makedirs(path, exist_ok=True)
    rank = _rank()
    flat = _flatten(state_dict)
    local = {}
    meta = {}
    for k, v in flat.items():
        if not isinstance(v, (Tensor, torch.Tensor)):
            meta[k] = {'value': v}
            continue
        gshape, off, owner = _local_region(v)
        t = (_unwrap(v) if isinstance(v, Tensor) else v).detach()
        if owner:
            local[k] = t.contiguous().cpu()
        meta[k] = {'global_shape': gshape, 'dtype': str(t.dtype).replace('torch.', ''),
                   'chunks': [{'rank': rank, 'offset': off, 'shape': list(t.shape)}] if owner else []}
    fname = f"{rank}_0.distcp"
    save_file(local, os.path.join(path, fname))
    metas = [None] * (dist.get_world_size() if dist.is_initialized() else 1)
    if dist.is_initialized():
        dist.all_gather_object(metas, meta, group=process_group)
    else:
        metas = [meta]
    if rank == coordinator_rank:
        merged = {}
        for r, m in enumerate(metas):
            for k, e in m.items():
                if 'value' in e:
                    merged.setdefault(k, {'value': e['value']})
                    continue
                ent = merged.setdefault(k, {'global_shape': e['global_shape'], 'dtype': e['dtype'], 'chunks': []})
                for c in e['chunks']:
                    c = dict(c, file=f"{c['rank']}_0.distcp")
                    ent['chunks'].append(c)
        with open(os.path.join(path, '0.metadata'), 'w') as f:
            json.dump({'state_dict_metadata': merged}, f)
    if dist.is_initialized():
        dist.barrier(group=process_group)


def load_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, offload=False):
    """Fills ``state_dict``'s tensors in place from a checkpoint saved with any sharding."""
    from safetensors import safe_open
    with open(os.path.join(path, '0.metadata')) as f:
        meta = json.load(f)['state_dict_metadata']
    flat = _flatten(state_dict)
    handles = {}

    def tensor_from(fname, key):
        if fname not in handles:
            handles[fname] = safe_open(os.path.join(path, fname), framework='pt')
        return handles[fname].get_tensor(key)

    for k, v in flat.items():
        if k not in meta or not isinstance(v, (Tensor, torch.Tensor)):
            continue
        ent = meta[k]
        dst = _unwrap(v) if isinstance(v, Tensor) else v
        gshape, off, _ = _local_region(v)
        want_lo, want_hi = off, [o + s for o, s in zip(off, dst.shape)]
        with torch.no_grad():
            for c in ent['chunks']:
                lo = c['offset']
                hi = [o + s for o, s in zip(lo, c['shape'])]
                ilo = [max(a, b) for a, b in zip(want_lo, lo)]
                ihi = [min(a, b) for a, b in zip(want_hi, hi)]
                if any(a >= b for a, b in zip(ilo, ihi)) and dst.dim() > 0:
                    continue
                src = tensor_from(c['file'], k)
                src_sl = tuple(slice(a - l_, b - l_) for a, b, l_ in zip(ilo, ihi, lo))
                dst_sl = tuple(slice(a - w, b - w) for a, b, w in zip(ilo, ihi, want_lo))
                dst[dst_sl].copy_(src[src_sl].to(dst.device, dst.dtype))
    for k, v in flat.items():
        if k in meta and 'value' in meta[k]:
            _set_nested(state_dict, k, meta[k]['value'])


def _set_nested(sd, key, value):
    parts = key.split('.')
    d = sd
    for p in parts[:-1]:
        if p in d and isinstance(d[p], dict):
            d = d[p]
        else:
            return
    if parts[-1] in d:
        d[parts[-1]] = value
