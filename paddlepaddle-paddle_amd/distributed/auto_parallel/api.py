"""Semi-automatic parallelism (reference: python/paddle/distributed/auto_parallel/api.py —
shard_tensor:131, dtensor_from_fn:545, reshard:579, shard_layer:678, ShardingStage1/2/3:1122+,
shard_optimizer:1353, Strategy:1583, DistModel:1864, to_static:2345, unshard_dtensor:2506,
shard_dataloader:2846; process_mesh.py ProcessMesh; placement_type.py Shard/Replicate/Partial).

A distributed tensor here is a paddle Tensor holding this rank's *local* piece plus its
``process_mesh``/``placements``/global shape.  ``reshard`` moves between placements with the
collective that is cheapest on point-to-point xGMI — Shard→Replicate all-gather, Partial→
Replicate all-reduce, Partial→Shard reduce-scatter, Shard(i)→Shard(j) all-to-all,
Replicate→Shard a local slice (no traffic) — each issued on the mesh-dimension subgroup.
"""
from ...framework.flags import pa_flag  # noqa: E402
import copy
import itertools

import numpy as np
import torch
import torch.distributed as dist

from ...core.tensor import Tensor, _wrap, _unwrap
from ...nn.layer.layers import Layer


# ----------------------------------------------------------------- placements
class Placement:
    def is_shard(self, dim=None):
        return False

    def is_replicated(self):
        return False

    def is_partial(self):
        return False


class Shard(Placement):
    def __init__(self, dim):
        self.dim = dim

    def get_dim(self):
        return self.dim

    def is_shard(self, dim=None):
        return dim is None or dim == self.dim

    def __eq__(self, o):
        return isinstance(o, Shard) and o.dim == self.dim

    def __hash__(self):
        return hash(('shard', self.dim))

    def __repr__(self):
        return f"Shard(dim={self.dim})"


class Replicate(Placement):
    def is_replicated(self):
        return True

    def __eq__(self, o):
        return isinstance(o, Replicate)

    def __hash__(self):
        return hash('replicate')

    def __repr__(self):
        return "Replicate()"


class ReduceType:
    kRedSum = 0
    kRedMax = 1
    kRedMin = 2
    kRedProd = 3
    kRedAvg = 4
    kRedAny = 5
    kRedAll = 6


class Partial(Placement):
    def __init__(self, reduce_type=ReduceType.kRedSum):
        self.reduce_type = reduce_type

    def is_partial(self):
        return True

    def __eq__(self, o):
        return isinstance(o, Partial) and o.reduce_type == self.reduce_type

    def __hash__(self):
        return hash(('partial', self.reduce_type))

    def __repr__(self):
        return f"Partial(reduce_type={self.reduce_type})"


# ----------------------------------------------------------------- mesh
_groups = {}


class ProcessMesh:
    def __init__(self, mesh=None, dim_names=None, shape=None, process_ids=None):
        if mesh is None:
            mesh = np.array(process_ids).reshape(shape)
        self._mesh = np.array(mesh)
        self._shape = list(self._mesh.shape)
        self._process_ids = self._mesh.reshape(-1).tolist()
        self._dim_names = list(dim_names) if dim_names is not None else [f"d{i}" for i in range(self._mesh.ndim)]

    @property
    def mesh(self):
        return self._mesh

    @property
    def shape(self):
        return list(self._shape)

    @property
    def ndim(self):
        return len(self._shape)

    @property
    def process_ids(self):
        return list(self._process_ids)

    @property
    def dim_names(self):
        return list(self._dim_names)

    def get_dim_size(self, dim):
        if isinstance(dim, str):
            dim = self._dim_names.index(dim)
        return self._shape[dim]

    def get_mesh_with_dim(self, dim_name, index=None):
        d = self._dim_names.index(dim_name)
        m = np.moveaxis(self._mesh, d, 0)
        names = [self._dim_names[d]] + [n for i, n in enumerate(self._dim_names) if i != d]
        if index is not None:
            return ProcessMesh(m[index], names[1:])
        return ProcessMesh(m, names)

    def coord(self, rank):
        idx = np.argwhere(self._mesh == rank)
        return tuple(idx[0]) if len(idx) else None

    def dim_group(self, dim, rank=None):
        """The process group along mesh dim ``dim`` containing ``rank``."""
        rank = dist.get_rank() if rank is None else rank
        c = self.coord(rank)
        sl = list(c)
        sl[dim] = slice(None)
        ranks = self._mesh[tuple(sl)].reshape(-1).tolist()
        return _subgroup(ranks), ranks

    def __contains__(self, rank):
        return rank in self._process_ids

    def __eq__(self, o):
        return isinstance(o, ProcessMesh) and np.array_equal(o._mesh, self._mesh) and o._dim_names == self._dim_names

    def __hash__(self):
        return hash((tuple(self._process_ids), tuple(self._shape)))

    def __repr__(self):
        return f"ProcessMesh(shape={self._shape}, process_ids={self._process_ids}, dim_names={self._dim_names})"


def _subgroup(ranks):
    """Subgroups are created collectively: the first time any mesh-dim group is requested,
    every rank creates the same set (all dims of all meshes seen so far are created on demand
    by the caller in a deterministic order)."""
    key = tuple(ranks)
    if key not in _groups:
        if dist.is_initialized() and len(ranks) == dist.get_world_size() and sorted(ranks) == list(range(len(ranks))):
            _groups[key] = None  # world group
        else:
            _groups[key] = dist.new_group(list(ranks)) if dist.is_initialized() else None
    return _groups[key]


def _ensure_mesh_groups(mesh):
    """Create every dim subgroup of ``mesh`` on every rank in a fixed order (new_group is collective)."""
    for d in range(mesh.ndim):
        other = [i for i in range(mesh.ndim) if i != d]
        for idx in itertools.product(*[range(mesh.shape[i]) for i in other]):
            sl = [slice(None)] * mesh.ndim
            for i, v in zip(other, idx):
                sl[i] = v
            _subgroup(mesh.mesh[tuple(sl)].reshape(-1).tolist())


# ----------------------------------------------------------------- dist tensors
class DistAttr:
    def __init__(self, mesh, sharding_specs):
        self.process_mesh = mesh
        self.sharding_specs = sharding_specs


def _local_slice(t, mesh, placements, rank):
    c = mesh.coord(rank)
    for d, p in enumerate(placements):
        if isinstance(p, Shard):
            n = mesh.shape[d]
            size = t.shape[p.dim]
            chunk = (size + n - 1) // n
            t = t.narrow(p.dim, min(c[d] * chunk, size), max(0, min(chunk, size - c[d] * chunk)))
    return t


def _attach(t, mesh, placements, global_shape):
    w = t if isinstance(t, Tensor) else _wrap(t)
    w.__dict__['process_mesh'] = mesh
    w.__dict__['placements'] = list(placements)
    w.__dict__['_global_shape'] = list(global_shape)
    w.__dict__['is_dist'] = lambda: True
    # the torch storage carries the dist attr too: ops see it through the SPMD mode
    # (auto_parallel_spmd: per-op sharding propagation + differentiable reshards)
    from .. import auto_parallel_spmd as spmd
    spmd.tag(w._t, mesh, placements, global_shape)
    if dist.is_initialized():
        spmd.enable()
    return w


def _dist_meta(t):
    """(mesh, placements, global_shape) of a dist tensor, from the handle or the storage tag."""
    if not isinstance(t, Tensor):
        return None
    if 'process_mesh' in t.__dict__:
        return t.__dict__['process_mesh'], t.__dict__['placements'], t.__dict__['_global_shape']
    from .. import auto_parallel_spmd as spmd
    return spmd.meta(t._t)


def is_dist_tensor(t):
    return _dist_meta(t) is not None


def _install_tensor_props():
    """Tensor.placements / process_mesh / is_dist() for tensors produced by SPMD-propagated ops
    (their dist attr lives on the storage tag; shard_tensor/reshard results also carry it on
    the handle)."""
    def _get(i, key):
        def f(self):
            d = self.__dict__
            if key in d:
                return d[key]
            m = _dist_meta(self)
            return m[i] if m else None
        return property(f)
    Tensor.process_mesh = _get(0, 'process_mesh')
    Tensor.placements = _get(1, 'placements')
    Tensor.is_dist = lambda self: _dist_meta(self) is not None


_install_tensor_props()


def shard_tensor(data, mesh, placements, dtype=None, place=None, stop_gradient=None):
    """``data`` is the global value (identical on every rank); returns this rank's local piece."""
    from ...core.tensor import to_tensor
    t = data if isinstance(data, Tensor) else to_tensor(data, dtype=dtype)
    _ensure_mesh_groups(mesh)
    g = _unwrap(t)
    rank = dist.get_rank() if dist.is_initialized() else 0
    local = _local_slice(g, mesh, placements, rank)
    for d, p in enumerate(placements):
        if isinstance(p, Partial) and mesh.coord(rank)[d] != 0:
            local = torch.zeros_like(local)  # partial: value lives on coordinate 0 of that dim
    out = _wrap(local.detach().clone().requires_grad_(g.requires_grad))
    if isinstance(t, Tensor) and hasattr(t, 'trainable'):
        from ...core.tensor import Parameter
        out = Parameter(out._t, trainable=not t.stop_gradient, name=t.name)
    if stop_gradient is not None:
        out.stop_gradient = stop_gradient
    return _attach(out, mesh, placements, g.shape)


def dtensor_from_fn(fn, mesh, placements, *args, **kwargs):
    return shard_tensor(fn(*args, **kwargs), mesh, placements)


def _red(rt):
    return {ReduceType.kRedSum: dist.ReduceOp.SUM, ReduceType.kRedMax: dist.ReduceOp.MAX,
            ReduceType.kRedMin: dist.ReduceOp.MIN, ReduceType.kRedProd: dist.ReduceOp.PRODUCT,
            ReduceType.kRedAvg: dist.ReduceOp.SUM}[rt]


def _all_gather_dim(t, group, n, dim):
    t = t.contiguous()
    if n == 1:
        return t
    parts = [torch.empty_like(t) for _ in range(n)]
    dist.all_gather(parts, t, group=group)
    return torch.cat(parts, dim)


def reshard(dist_tensor, mesh, placements):
    t = _unwrap(dist_tensor)
    m = _dist_meta(dist_tensor)
    src_mesh = m[0] if m else mesh
    src = list(m[1]) if m else [Replicate()] * mesh.ndim
    gshape = list(m[2]) if m else list(t.shape)
    if src_mesh == mesh and t.requires_grad and torch.is_grad_enabled():
        # differentiable path: conjugate collectives in backward
        from .. import auto_parallel_spmd as spmd
        _ensure_mesh_groups(mesh)
        return _attach(_wrap(spmd._reshard_local(t, mesh, src, list(placements))), mesh, placements, gshape)
    if src_mesh != mesh:
        # cross-mesh: materialise the global value then re-slice (all ranks participate)
        full = unshard_dtensor(dist_tensor)
        return shard_tensor(full, mesh, placements)
    _ensure_mesh_groups(mesh)
    rank = dist.get_rank() if dist.is_initialized() else 0
    cur = t
    for d in range(mesh.ndim):
        s, dst = src[d], placements[d]
        if s == dst:
            continue
        grp, ranks = mesh.dim_group(d, rank)
        n = len(ranks)
        if isinstance(s, Partial):
            cur = cur.contiguous().clone()  # collectives below work in place; never touch the source
            if isinstance(dst, Shard):
                # reduce-scatter along dst.dim
                chunks = list(cur.chunk(n, dst.dim))
                out = torch.empty_like(chunks[ranks.index(rank)].contiguous())
                dist.reduce_scatter(out, [c.contiguous() for c in chunks], op=_red(s.reduce_type), group=grp)
                cur = out
            else:
                dist.all_reduce(cur, op=_red(s.reduce_type), group=grp)
                if s.reduce_type == ReduceType.kRedAvg:
                    cur = cur / n
        elif isinstance(s, Shard):
            if isinstance(dst, Replicate):
                cur = _all_gather_dim(cur, grp, n, s.dim)
            elif isinstance(dst, Shard):
                # Shard(i) -> Shard(j): all-to-all
                ins = [c.contiguous() for c in cur.chunk(n, dst.dim)]
                outs = [torch.empty_like(ins[0]) for _ in range(n)]
                from ..communication import all_to_all_tensors
                all_to_all_tensors(outs, ins, grp)
                cur = torch.cat(outs, s.dim)
            else:  # Shard -> Partial: keep on coordinate 0 after gathering
                cur = _all_gather_dim(cur, grp, n, s.dim)
                if ranks.index(rank) != 0:
                    cur = torch.zeros_like(cur)
        else:  # Replicate ->
            if isinstance(dst, Shard):
                size = cur.shape[dst.dim]
                chunk = (size + n - 1) // n
                i = ranks.index(rank)
                cur = cur.narrow(dst.dim, min(i * chunk, size), max(0, min(chunk, size - i * chunk)))
            elif isinstance(dst, Partial):
                if ranks.index(rank) != 0:
                    cur = torch.zeros_like(cur)
        src[d] = dst
    return _attach(_wrap(cur), mesh, placements, gshape)


def unshard_dtensor(dist_tensor):
    m = _dist_meta(dist_tensor)
    mesh = m[0] if m else None
    if mesh is None:
        return dist_tensor
    r = reshard(dist_tensor, mesh, [Replicate()] * mesh.ndim)
    out = _wrap(_unwrap(r))
    return out


# ----------------------------------------------------------------- layers / optimizers / data
def shard_layer(layer, process_mesh, shard_fn=None, input_fn=None, output_fn=None):
    """Calls ``shard_fn(name, sublayer, mesh)`` for every sublayer (default: replicate all
    parameters), then wires optional input/output resharding hooks."""
    def replicate_all(name, sub, mesh):
        for pname, p in list(sub._parameters.items()):
            if p is not None and not is_dist_tensor(p):
                sub._parameters[pname] = shard_tensor(p, mesh, [Replicate()] * mesh.ndim)
    fn = shard_fn or replicate_all
    for name, sub in layer.named_sublayers(include_self=True):
        fn(name, sub, process_mesh)
    if shard_fn is not None:
        for name, sub in layer.named_sublayers(include_self=True):
            replicate_all(name, sub, process_mesh)
    if input_fn is not None:
        layer.register_forward_pre_hook(lambda lyr, inp: input_fn(inp, process_mesh))
    if output_fn is not None:
        layer.register_forward_post_hook(lambda lyr, inp, out: output_fn(out, process_mesh))
    return layer


class _ShardingStageBase:
    """Reference python/paddle/distributed/auto_parallel/api.py ShardingStage1/2/3: passed to
    shard_optimizer, it partitions the optimizer state (stage 1), also the gradients (stage 2)
    and also the parameters (stage 3) over one mesh dimension."""
    level = None

    def __init__(self, mesh=None, sharding_mesh_dim=None):
        self._mesh = mesh
        self._sharding_mesh_dim = sharding_mesh_dim

    def _group(self, params):
        """Process group of the sharding axis: ``sharding_mesh_dim`` of the mesh (default: the
        mesh of the first parameter, its dim 0, i.e. the data-parallel axis), or the world."""
        mesh = self._mesh
        if mesh is None:
            for p in params:
                m = _dist_meta(p)
                if m is not None:
                    mesh = m[0]
                    break
        if mesh is None or not dist.is_initialized():
            return None
        d = self._sharding_mesh_dim
        if isinstance(d, str):
            d = mesh.dim_names.index(d)
        d = 0 if d is None else int(d)
        _ensure_mesh_groups(mesh)
        grp, _ = mesh.dim_group(d)
        return grp


class ShardingStage1(_ShardingStageBase):
    level = 'os'


class ShardingStage2(_ShardingStageBase):
    level = 'os_g'


class ShardingStage3(_ShardingStageBase):
    level = 'p_g_os'


class _ShardOptimizer:
    """shard_optimizer result.

    * no shard_fn: gradients of parameters replicated along a mesh dim are averaged over that
      dim with ONE coalesced all-reduce per (dim group, dtype) bucket (not one call per
      parameter), then the wrapped optimizer steps.
    * ShardingStage1/2: a sharding engine (parallel/sharding.py, the same one as fleet's
      DygraphShardingOptimizer) over the sharding-axis group owns the optimizer: gradients are
      reduce-scattered asynchronously as they land in backward, each rank updates its shard of the
      fp32 master / moments with the fused kernel, parameters are all-gathered after the step.
    * ShardingStage3: the same, plus the parameters themselves are released between uses when the
      model is known (dist.to_static / DistModel passes its layer); a bare optimizer gets stage-2
      behaviour.
    """

    def __init__(self, optimizer, shard_fn=None, layer=None, gradient_accumulation_steps=1, engine_kwargs=None):
        self._inner_opt = optimizer
        self._shard_fn = shard_fn
        self._engine = None
        self._sharded = None
        # gradient accumulation (reference: shard_optimizer(..., gradient_accumulation_steps)):
        # step() / clear_grad() act on every k-th call; the k-1 calls in between leave the
        # accumulated gradients in place
        self._acc_k = max(1, int(gradient_accumulation_steps))
        self._acc_n = 0
        if shard_fn is not None:
            if not isinstance(shard_fn, _ShardingStageBase):
                raise TypeError("shard_fn must be a ShardingStage1/2/3 instance")
            from ...parallel.sharding import ShardingEngine, ShardedOptimizer
            params = [p for p in optimizer._parameter_list if not p.stop_gradient]
            grp = shard_fn._group(params)
            level = shard_fn.level
            if level == 'p_g_os' and layer is None:
                level = 'os_g'
            kw = dict(engine_kwargs or {})
            if level == 'p_g_os':
                self._engine = ShardingEngine(layer, level, group=grp, **kw)
            else:
                self._engine = ShardingEngine(None, level, group=grp, params=params)
            self._sharded = ShardedOptimizer(optimizer, self._engine)

    def _sync_grads(self):
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors
        buckets = {}
        for p in self._inner_opt._parameter_list:
            g = p._t.grad
            if g is None:
                continue
            m = _dist_meta(p)
            mesh, pl = (m[0], m[1]) if m else (None, None)
            if mesh is None:
                buckets.setdefault((tuple(range(dist.get_world_size())), g.dtype), [None, []])[1].append(g)
                continue
            for d, pd in enumerate(pl):
                if isinstance(pd, Replicate) and mesh.shape[d] > 1:
                    grp, ranks = mesh.dim_group(d)
                    b = buckets.setdefault((tuple(ranks), g.dtype), [grp, []])
                    b[1].append(g)
        for (ranks, dt), (grp, gs) in buckets.items():
            flat = _flatten_dense_tensors(gs)
            dist.all_reduce(flat, group=grp)
            flat.div_(len(ranks))
            for g, r in zip(gs, _unflatten_dense_tensors(flat, gs)):
                g.copy_(r)

    def _boundary(self):
        return self._acc_n % self._acc_k == 0

    def step(self):
        self._acc_n += 1
        if not self._boundary():
            return None
        if self._sharded is not None:
            return self._sharded.step()
        self._sync_grads()
        self._inner_opt.step()

    def clear_grad(self, set_to_zero=True):
        if not self._boundary():
            return None  # mid-accumulation: keep the summed gradients
        if self._sharded is not None:
            return self._sharded.clear_grad()
        self._inner_opt.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def state_dict(self):
        return self._sharded.state_dict() if self._sharded is not None else self._inner_opt.state_dict()

    def set_state_dict(self, sd):
        if self._sharded is not None:
            return self._sharded.set_state_dict(sd)
        return self._inner_opt.set_state_dict(sd)

    def __getattr__(self, name):
        return getattr(self._inner_opt, name)


def shard_optimizer(optimizer, shard_fn=None, gradient_accumulation_steps=1):
    return _ShardOptimizer(optimizer, shard_fn, gradient_accumulation_steps=gradient_accumulation_steps)



def shard_scaler(scaler):
    """Reference api.py shard_scaler: the found-inf decision is all-reduced (MAX) over every rank,
    so ranks holding different shards skip or apply the step together."""
    def sync(found):
        v = float(found) if isinstance(found, bool) else float(found.item() > 0)
        if dist.is_initialized() and dist.get_world_size() > 1:
            import torch as _t
            dev = _t.device('cuda', _t.cuda.current_device()) if (_t.cuda.is_available() and
                                                                 dist.get_backend() == 'nccl') else _t.device('cpu')
            t = _t.tensor([v], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            v = float(t.item())
        return v > 0
    scaler._sync_found_inf = sync
    return scaler


class _ShardDataLoader:
    def __init__(self, loader, meshes, input_keys=None, shard_dims=None, is_dataset_splitted=False):
        self._loader = loader
        self._meshes = meshes if isinstance(meshes, (list, tuple)) else [meshes]
        self._shard_dims = shard_dims
        self._split = is_dataset_splitted

    def __len__(self):
        return len(self._loader)

    def __iter__(self):
        mesh = self._meshes[0]
        dim = self._shard_dims if isinstance(self._shard_dims, int) else 0
        if isinstance(self._shard_dims, str):
            dim = mesh.dim_names.index(self._shard_dims)
        for batch in self._loader:
            if self._split or not dist.is_initialized():
                yield batch
                continue
            pl = [Replicate()] * mesh.ndim
            pl[dim] = Shard(0)
            items = batch if isinstance(batch, (list, tuple)) else [batch]
            out = [shard_tensor(b, mesh, pl) if isinstance(b, Tensor) else b for b in items]
            yield out if isinstance(batch, (list, tuple)) else out[0]


def shard_dataloader(dataloader, meshes, input_keys=None, shard_dims=None, is_dataset_splitted=False):
    return _ShardDataLoader(dataloader, meshes, input_keys, shard_dims, is_dataset_splitted)


class Strategy:
    """Config groups mirroring the reference's auto-parallel Strategy."""

    class _Cfg(dict):
        __getattr__ = dict.get

        def __setattr__(self, k, v):
            self[k] = v

    def __init__(self, config=None):
        config = config or {}

        def cfg(name, **defaults):
            c = Strategy._Cfg(defaults)
            c.update(config.get(name, {}))
            return c
        self.sharding = cfg('sharding', enable=False, stage=1, degree=8)
        self.gradient_merge = cfg('gradient_merge', enable=False, k_steps=1, avg=True)
        self.pipeline = cfg('pipeline', enable=False, schedule_mode='1F1B', micro_batch_size=1, accumulate_steps=1)
        self.amp = cfg('amp', enable=False, dtype='bfloat16', level='O2')
        self.recompute = cfg('recompute', enable=False)
        self.fused_passes = cfg('fused_passes', enable=False, fused_passes_list=[])
        # 'semi': the user's placements; 'full': the rule-based planner places the parameters
        # (auto_parallel/static/planner.py) on get_mesh() at the first step
        self.auto_mode = config.get('auto_mode', 'semi')


_GLOBAL_MESH = [None]


def set_mesh(mesh):
    """The default process mesh of auto-parallel APIs (the fully automatic planner uses it)."""
    _GLOBAL_MESH[0] = mesh


def get_mesh():
    return _GLOBAL_MESH[0]


class DistModel:
    """``dist.to_static`` result: ``train()/eval()/predict()`` switch the mode; calling it runs
    one step (forward + loss + backward + update in train mode)."""

    def __init__(self, layer, loader, loss=None, optimizer=None, strategy=None, metrics=None):
        self._layer = layer
        self._loader = loader
        self._loss = loss
        self._strategy = strategy or Strategy()
        st = self._strategy
        # sharding: optimizer states (and grads / params by stage) over the data-parallel axis
        if optimizer is not None and st.sharding.get('enable'):
            inner = optimizer._inner_opt if isinstance(optimizer, _ShardOptimizer) else optimizer
            stage = {1: ShardingStage1, 2: ShardingStage2, 3: ShardingStage3}[int(st.sharding.get('stage', 1))]()
            acc = optimizer._acc_k if isinstance(optimizer, _ShardOptimizer) else 1
            kw = {}
            if st.sharding.get('segment_size') is not None:  # stage 3: units below this stay materialised
                kw['segment_size'] = int(st.sharding.get('segment_size'))
            optimizer = _ShardOptimizer(inner, stage, layer=layer, gradient_accumulation_steps=acc, engine_kwargs=kw)
        self._opt = optimizer
        # pipeline: one call = one mini-batch of ``accumulate_steps`` micro-batches (or
        # batch / micro_batch_size of them), run in the configured schedule's order and followed by
        # ONE optimizer update; stage placement across meshes runs through the SPMD reshards
        pp = st.pipeline
        self._pp = bool(pp.get('enable'))
        self._pp_acc = max(1, int(pp.get('accumulate_steps', 1) or 1))
        self._pp_mbs = int(pp.get('micro_batch_size', 1) or 1)
        self._pp_mode = str(pp.get('schedule_mode', '1F1B'))
        gm = st.gradient_merge
        self._k = int(gm.get('k_steps', 1)) if gm.get('enable') else 1
        self._avg = bool(gm.get('avg', True))
        self._micro = 0
        if st.recompute.get('enable'):
            from ..fleet.recompute import recompute

            def wrap(f):
                return lambda *a, **k: recompute(f, *a, **k) if layer.training else f(*a, **k)
            for _, sub in list(layer.named_children()):
                sub.forward = wrap(sub.forward)
        self._mode = 'train' if optimizer is not None and loss is not None else 'predict'
        # pipeline stages from the process meshes the parameters were placed on (shard_layer /
        # shard_tensor with Replicate placements, one mesh per stage, in forward order)
        self._pp_plan = self._pipeline_plan(layer) if self._pp else None
        self._pp_stale = False
        # static form: the step is recorded once per (mode, input signature) into a static
        # Program and replayed by the Executor (reference: to_static builds the distributed
        # program); the eager step remains for what the program form does not cover
        self._static_reason = self._static_blocker(layer, optimizer, st)
        self._progs = {}
        self._exe = None
        self._auto_pending = (getattr(st, 'auto_mode', 'semi') == 'full' and dist.is_initialized()
                              and dist.get_world_size() > 1
                              and all(_dist_meta(p) is None for p in layer.parameters()))
        self.plan = None

    def _auto_plan(self, args):
        """auto_mode 'full': place the parameters by the rule-based planner (reference
        static/planner_v2.py + tuner/rule_based_tuner.py), then build the step as usual."""
        from .static.planner import RuleBasedPlanner
        mesh = get_mesh() or ProcessMesh(list(range(dist.get_world_size())), dim_names=['mp'])
        inputs = args if self._mode == 'predict' else args[:-1]
        planner = RuleBasedPlanner(mesh)
        was = self._layer.training
        self._layer.eval()  # plan on the inference graph (no dropout nodes)
        try:
            self.plan = planner.plan(self._layer, *inputs)
        finally:
            if was:
                self._layer.train()
        planner.apply(self._layer, self.plan, self._opt)
        self._auto_pending = False
        self._static_reason = self._static_blocker(self._layer, self._opt, self._strategy)
        self._progs = {}

    @staticmethod
    def _static_blocker(layer, optimizer, st):
        """None when the step can run as a static Program, else why it runs eagerly."""
        import os
        if not pa_flag('dist_to_static'):
            return 'disabled by PADDLE_AMD_DIST_TO_STATIC=0'
        sharded = isinstance(optimizer, _ShardOptimizer) and optimizer._sharded is not None
        if st.pipeline.get('enable'):
            if DistModel._pipeline_plan(layer) is None:
                return 'pipeline stages need the parameters placed on one process mesh per stage'
            if sharded:
                return 'sharding inside pipeline stages runs eagerly'
        if sharded and st.amp.get('enable'):
            return 'AMP over a sharded optimizer runs eagerly'
        tp = any(m is not None and any(not isinstance(x, Replicate) for x in m[1])
                 for m in (_dist_meta(p) for p in layer.parameters()))
        if tp and (st.pipeline.get('enable') or sharded):
            return 'tensor-parallel placements with pipeline / sharding run on the SPMD-propagated eager path'
        return None

    @staticmethod
    def _pipeline_plan(layer):
        """{'meshes': stage meshes, 'layer_stage': {id(sublayer): stage}} from the parameters'
        process meshes (Replicate placements only), or None when fewer than two stages are marked
        or the stage meshes differ in size."""
        meshes, layer_stage = [], {}
        for sub in layer.sublayers(include_self=True):
            own = [q for q in sub._parameters.values() if q is not None]
            for q in own:
                m = _dist_meta(q)
                if m is None:
                    continue
                if any(not isinstance(x, Replicate) for x in m[1]):
                    return None
                if m[0] not in meshes:
                    meshes.append(m[0])
                layer_stage[id(sub)] = meshes.index(m[0])
                break
        if len(meshes) < 2 or len({len(m.process_ids) for m in meshes}) != 1:
            return None
        return {'meshes': meshes, 'layer_stage': layer_stage}

    def _pipeline_config(self):
        """static/pipeline.PipelineConfig of this rank (stage = the mesh holding it; the j-th
        rank of every stage mesh forms one pipe; the ranks of a stage mesh are its data-parallel
        replicas) and the data-parallel group of the stage."""
        import types
        from ...static.pipeline import PipelineConfig
        meshes = self._pp_plan['meshes']
        rank = dist.get_rank() if dist.is_initialized() else 0
        stage = next(k for k, m in enumerate(meshes) if rank in m)
        j = meshes[stage].process_ids.index(rank)
        pipe = [m.process_ids[j] for m in meshes]
        for m in meshes:  # every rank creates the same groups in the same order (new_group is collective)
            _subgroup(m.process_ids)
        for jj in range(len(meshes[0].process_ids)):
            _subgroup([m.process_ids[jj] for m in meshes])
        grp = types.SimpleNamespace(ranks=pipe, pg=_subgroup(pipe))
        S = len(meshes)
        cfg = PipelineConfig(stage, S, self._pp_acc, grp, pipe[stage - 1] if stage > 0 else None,
                             pipe[stage + 1] if stage < S - 1 else None, self._pp_mode)
        dpr = meshes[stage].process_ids
        dp = types.SimpleNamespace(pg=_subgroup(dpr), nranks=len(dpr), ranks=dpr) if len(dpr) > 1 else None
        return cfg, dp

    def _sync_stage_params(self):
        """Every stage's parameters from the first rank of its mesh to all ranks (each rank updates
        only its own stage's copy in training; a whole-model eval / predict needs all of them)."""
        if not self._pp_stale or not dist.is_initialized():
            return
        import torch as _t
        meshes, ls = self._pp_plan['meshes'], self._pp_plan['layer_stage']
        with _t.no_grad():
            for sub in self._layer.sublayers(include_self=True):
                if id(sub) not in ls:
                    continue
                src = meshes[ls[id(sub)]].process_ids[0]
                for q in sub._parameters.values():
                    if q is not None:
                        dist.broadcast(_unwrap(q), src)
        self._pp_stale = False

    @property
    def is_static(self):
        return self._static_reason is None

    def _dp_of(self, args):
        """Data-parallel group of the step: the mesh dim the inputs' batch axis is sharded on."""
        for a in args:
            m = _dist_meta(a)
            if m is None:
                continue
            mesh, placements, _ = m
            for d, p in enumerate(placements):
                if isinstance(p, Shard) and p.dim == 0 and mesh.shape[d] > 1:
                    _ensure_mesh_groups(mesh)
                    rank = dist.get_rank() if dist.is_initialized() else 0
                    c = mesh.coord(rank)
                    sl = [c[i] if i != d else slice(None) for i in range(mesh.ndim)]
                    ranks = mesh.mesh[tuple(sl)].reshape(-1).tolist()
                    import types
                    return types.SimpleNamespace(pg=_subgroup(ranks), nranks=len(ranks))
        return None

    def _build_static(self, mode, args):
        import torch as _t
        from ... import static as _st
        from ...static.program import _static_minimize
        from ...static.minimize import step_policy
        from ... import framework as _fw
        from ...static import program as _prog
        vals = [_unwrap(a) if isinstance(a, Tensor) else _t.as_tensor(a) for a in args]
        was_dynamic = _fw.in_dynamic_mode()
        if was_dynamic:
            _fw.enable_static()
        from .. import auto_parallel_spmd as spmd
        spmd_on = spmd._mode[0] is not None
        if spmd_on:
            # SPMD propagation above the recorder: it sees the global-view ops and hands the
            # recorder the per-shard ops plus one node per reshard collective
            spmd.disable()
            _prog._stop_recording()
            _prog._start_recording()
            spmd.enable()
        pp = self._pp_plan if (mode == 'train' and self._pp_plan is not None) else None
        hooks = []
        if pp is not None:  # ops recorded inside a stage's sublayers run on that stage
            for sub in self._layer.sublayers(include_self=True):
                k = pp['layer_stage'].get(id(sub))
                if k is not None:
                    hooks.append(sub.register_forward_pre_hook(
                        lambda lyr, inp, _k=k: _prog._STAGE.__setitem__(0, _k)))
        prev_stage = _prog._STAGE[0]
        eng = self._opt._engine if isinstance(self._opt, _ShardOptimizer) else None
        if eng is not None:
            eng.hooks_off = True  # stage 3: recording gathers nothing; the replay is gathered up front
        try:
            main, startup = _st.Program(), _st.Program()
            with _st.program_guard(main, startup):
                dt_name = {_t.float32: 'float32', _t.float16: 'float16', _t.bfloat16: 'bfloat16', _t.int64: 'int64',
                           _t.int32: 'int32', _t.float64: 'float64', _t.bool: 'bool', _t.uint8: 'uint8'}
                feeds = [_st.data(f'dm_input_{i}', [-1] + list(v.shape[1:]), dt_name[v.dtype])
                         for i, v in enumerate(vals)]
                amp = self._strategy.amp
                import contextlib
                if amp.get('enable') and mode != 'train':
                    from ...amp import auto_cast
                    ctx = auto_cast(True, level=amp.get('level', 'O2'), dtype=amp.get('dtype', 'bfloat16'))
                else:
                    ctx = contextlib.nullcontext()
                if mode == 'predict':
                    with ctx:
                        fetch = self._layer(*feeds)
                else:
                    with ctx:
                        out = self._layer(*feeds[:-1])
                        if pp is not None:
                            _prog._STAGE[0] = len(pp['meshes']) - 1  # the loss: last stage
                        fetch = self._loss(out, feeds[-1])
                    if mode == 'train':
                        opt = self._opt
                        if isinstance(opt, _ShardOptimizer):
                            opt = opt._sharded if opt._sharded is not None else opt._inner_opt
                        if amp.get('enable'):
                            from ...static import amp as samp
                            dtype = amp.get('dtype', 'bfloat16')
                            lists = samp.AutoMixedPrecisionLists(custom_white_list=amp.get('custom_white_list'),
                                                                 custom_black_list=amp.get('custom_black_list'),
                                                                 dtype=dtype)
                            opt = samp.decorate(opt, amp_lists=lists, level=amp.get('level', 'O2'), dtype=dtype)
                            opt.minimize(fetch)
                        else:
                            _static_minimize(opt, fetch)
                        pol = step_policy(main)
                        acc = self._opt._acc_k if isinstance(self._opt, _ShardOptimizer) else 1
                        pol.k_steps, pol.avg = self._k * acc, (self._avg if acc == 1 or self._k > 1 else False)
                        # a sharded optimizer averages its gradients in its reduce-scatter
                        sharded = isinstance(self._opt, _ShardOptimizer) and self._opt._sharded is not None
                        pol.dp_group = None if sharded else self._dp_of(args)
                        if pp is not None:
                            pol.pipeline, pol.dp_group = self._pipeline_config()
        finally:
            _prog._STAGE[0] = prev_stage
            for h in hooks:
                h.remove()
            if eng is not None:
                eng.hooks_off = False
            if spmd_on:
                spmd.disable()  # modes leave LIFO: SPMD first, the recorder with static mode
            if was_dynamic:
                _fw.disable_static()
            if spmd_on:
                spmd.enable()
        if self._exe is None:
            self._exe = _st.Executor()
        plan = (main, [f'dm_input_{i}' for i in range(len(vals))], fetch, self._dp_of(args))
        return plan

    def _static_call(self, args):
        import torch as _t
        key = (self._mode, tuple((tuple(_unwrap(a).shape[1:]), _unwrap(a).dtype) if isinstance(a, Tensor)
                                 else (type(a),) for a in args))
        plan = self._progs.get(key)
        if plan is None:
            plan = self._progs[key] = self._build_static(self._mode, args)
        prog, names, fetch, dp = plan
        feed = {n: (_unwrap(a).detach() if isinstance(a, Tensor) else a) for n, a in zip(names, args)}
        eng = self._opt._engine if isinstance(self._opt, _ShardOptimizer) else None
        if eng is not None and eng.level == 3:
            # stage 3 in the program form: every unit is gathered for the step (its gradient
            # reduce-scattered as it completes in backward) and released again after it
            for u in eng.units:
                u.wait_gather()
                if self._mode == 'train':
                    u.alloc_grads()
        if self._pp_plan is not None:
            if self._mode == 'train':
                self._pp_stale = True
            else:
                self._sync_stage_params()
        from .. import auto_parallel_spmd as spmd
        spmd_on = spmd._mode[0] is not None
        if spmd_on:
            spmd.disable()  # the program already holds the per-shard ops and reshards
        try:
            res = self._exe.run(prog, feed=feed, fetch_list=[fetch], return_numpy=False)[0]
        finally:
            if spmd_on:
                spmd.enable()
        if eng is not None and eng.level == 3 and self._mode != 'train':
            for u in eng.units:
                u.free_params()
        if self._mode != 'predict' and dp is not None and self._pp_plan is None:
            # the loss of the global batch: the mean of the data-parallel ranks' local losses
            r = _unwrap(res).detach().float().clone()
            dist.all_reduce(r, group=dp.pg)
            res = _wrap((r / dp.nranks).to(_unwrap(res).dtype))
        return res

    def train(self):
        self._mode = 'train'
        self._layer.train()

    def eval(self):
        self._mode = 'eval'
        self._layer.eval()

    def predict(self):
        self._mode = 'predict'
        self._layer.eval()

    def __call__(self, *args):
        if self._auto_pending:
            self._auto_plan(args)
        if self._static_reason is None:
            return self._static_call(args)
        if self._mode == 'predict':
            import torch as _t
            with _t.no_grad():
                return self._layer(*args)
        inputs, labels = args[:-1], args[-1]
        amp = self._strategy.amp
        if amp.get('enable'):
            from ...amp import auto_cast
            ctx = auto_cast(True, custom_white_list=amp.get('custom_white_list'),
                            custom_black_list=amp.get('custom_black_list'), level=amp.get('level', 'O2'),
                            dtype=amp.get('dtype', 'bfloat16'))
        else:
            import contextlib
            ctx = contextlib.nullcontext()
        if self._pp and self._mode == 'train':
            return self._pipeline_step(inputs, labels, ctx)
        with ctx:
            out = self._layer(*inputs)
            loss = self._loss(out, labels)
        if self._mode == 'train':
            # gradient merge: k micro-steps accumulate before one update ('avg' divides by k)
            (loss / self._k if (self._k > 1 and self._avg) else loss).backward()
            self._micro += 1
            if self._micro % self._k == 0:
                self._opt.step()
                self._opt.clear_grad()
        return loss

    def _micro_batches(self, inputs, labels):
        lead = labels if isinstance(labels, Tensor) else next((x for x in inputs if isinstance(x, Tensor)), None)
        B = lead.shape[0] if lead is not None else 1
        n = self._pp_acc if self._pp_acc > 1 else max(1, B // max(1, self._pp_mbs))
        if B % n:
            raise ValueError(f"pipeline: batch {B} does not split into {n} micro-batches")
        m = B // n

        def cut(x, i):
            return x[i * m:(i + 1) * m] if isinstance(x, Tensor) and x.shape and x.shape[0] == B else x
        return [([cut(x, i) for x in inputs], cut(labels, i)) for i in range(n)]

    def _pipeline_step(self, inputs, labels, ctx):
        """Micro-batched step (reference auto-parallel pipeline: accumulate_steps micro-batches per
        mini-batch, schedule FThenB / 1F1B / VPP).  Every micro-batch's loss is scaled by 1/n and its
        gradients accumulate; the update runs once.  FThenB runs all forwards before the backwards
        (activations of every micro-batch alive), 1F1B interleaves (one micro-batch in flight)."""
        mbs = self._micro_batches(inputs, labels)
        n = len(mbs)
        losses = []
        if self._pp_mode.upper() == 'FTHENB':
            pending = []
            for x, y in mbs:
                with ctx:
                    loss = self._loss(self._layer(*x), y)
                pending.append(loss)
            for loss in pending:
                (loss / n).backward()
                losses.append(loss.detach())
        else:
            for x, y in mbs:
                with ctx:
                    loss = self._loss(self._layer(*x), y)
                (loss / n).backward()
                losses.append(loss.detach())
        self._micro += 1
        if self._micro % self._k == 0:
            self._opt.step()
            self._opt.clear_grad()
        from ...tensor.manipulation import stack
        return stack(losses).mean()

    def _materialize(self):
        """Stage 3: gather every released unit (the parameters a state dict reads)."""
        eng = self._opt._engine if isinstance(self._opt, _ShardOptimizer) else None
        if eng is not None and eng.level == 3:
            for u in eng.units:
                u.wait_gather()

    def state_dict(self, mode='all'):
        self._materialize()
        sd = dict(self._layer.state_dict())
        if mode in ('all', 'opt') and self._opt is not None:
            sd.update(self._opt.state_dict())
        return sd

    def set_state_dict(self, state_dict):
        self._layer.set_state_dict(state_dict)

    # ---- the distributed programs (reference api.py:2010-2068 DistModel.dist_main_program /
    # dist_startup_program). The program of a mode is recorded at its first call: the per-shard
    # ops plus one node per reshard collective, every value tagged with its dist attribute
    # (``Program.dist_attr``). Parameters are created already placed (shard_tensor /
    # shard_layer), so the startup program holds no initializers.
    def _prog_for(self, mode):
        mode = mode or self._mode
        progs = [p for (m, _), p in self._progs.items() if m == mode]
        return progs[-1][0] if progs else None

    def dist_main_program(self, mode=None):
        """The recorded distributed Program of ``mode`` (default: the current one); None before
        that mode has run a step."""
        return self._prog_for(mode)

    def dist_startup_program(self, mode=None):
        from ... import static as _st
        return _st.Program() if self._prog_for(mode) is not None else None

    def serial_startup_program(self, mode=None):
        """Parameters are created eagerly (then placed), so the serial startup program is empty."""
        from ... import static as _st
        return _st.Program() if self._prog_for(mode) is not None else None

    def serial_main_program(self, mode=None):
        """The unpartitioned step of ``mode`` for analysis (reference api.py:2049): the forward (and
        the loss outside 'predict') recorded with SPMD propagation off and every placed parameter at
        its GLOBAL shape — its Program constant is a meta tensor of that shape, so the program is
        an op graph to inspect, not to run.  None before that mode has run a step."""
        import torch as _t
        from ... import static as _st
        from ... import framework as _fw
        from .. import auto_parallel_spmd as spmd
        mode = mode or self._mode
        keys = [k for k in self._progs if k[0] == mode]
        if not keys or any(len(s) != 2 for s in keys[-1][1]):
            return None
        specs = keys[-1][1]
        dt_name = {_t.float32: 'float32', _t.float16: 'float16', _t.bfloat16: 'bfloat16', _t.int64: 'int64',
                   _t.int32: 'int32', _t.float64: 'float64', _t.bool: 'bool', _t.uint8: 'uint8'}
        main = _st.Program()
        was_dynamic = _fw.in_dynamic_mode()
        spmd_on = spmd._mode[0] is not None
        if spmd_on:
            spmd.disable()
        if was_dynamic:
            _fw.enable_static()
        try:
            for p in self._layer.parameters():
                m = spmd.meta(p._t)
                if m is not None:  # a placed parameter: its global-shape twin
                    cid = main._const(p._t, owner=p)
                    twin = _t.empty(list(m[2]), dtype=p._t.dtype, device='meta')
                    if p._t.requires_grad:
                        twin.requires_grad_(True)
                    main._meta_twins[cid] = twin
            with _st.program_guard(main, _st.Program()):
                feeds = [_st.data(f'dm_input_{i}', [-1] + list(shape), dt_name[dtype])
                         for i, (shape, dtype) in enumerate(specs)]
                if mode == 'predict':
                    self._layer(*feeds)
                else:
                    self._loss(self._layer(*feeds[:-1]), feeds[-1])
        finally:
            if was_dynamic:
                _fw.disable_static()
            if spmd_on:
                spmd.enable()
        return main


def to_static(layer, loader=None, loss=None, optimizer=None, strategy=None, input_spec=None):
    return DistModel(layer, loader, loss, optimizer, strategy)


_ = (copy, Layer)


# the high-level Engine lives in auto_parallel/static/engine.py (reference layout)
def __getattr__(name):
    if name == 'Engine':
        from .static.engine import Engine
        return Engine
    raise AttributeError(name)
