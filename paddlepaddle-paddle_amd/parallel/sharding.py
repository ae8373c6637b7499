"""Group-sharded data parallelism (ZeRO) stage 1 / 2 / 3 over RCCL.

Reference: python/paddle/distributed/sharding/group_sharded.py (group_sharded_parallel),
python/paddle/distributed/fleet/meta_parallel/sharding/group_sharded_stage2.py,
group_sharded_stage3.py:85 (GroupShardedStage3), group_sharded_optimizer_stage2.py.

MI355X design — everything is a contiguous slice:

* A **unit** is a FlatBuffer of parameters padded to a multiple of (world × 64) elements.
  Rank r owns elements [r·L, (r+1)·L) of every unit (L = numel / world).
  - stage 1/2 ('os', 'os_g'): units are ~``bucket_mb`` slices of one flat buffer per dtype;
    parameters stay materialised on every rank.
  - stage 3 ('p_g_os'): one unit per layer block (greedy split of the layer tree at
    ``segment_size`` elements); a unit's full parameter storage exists only while the block
    runs forward or backward (storage resize to 0 otherwise), gathered by one
    ``all_gather_into_tensor`` per unit with the next unit's gather prefetched
    asynchronously; embedding units are kept materialised (their weights are commonly tied
    to the LM head and used outside their own layer).
* Gradients accumulate into per-unit flat buffers; the moment a unit's last gradient lands a
  ``reduce_scatter_tensor`` (AVG) of the whole unit is launched asynchronously, so it
  overlaps the backward of earlier units.  Stage 3 materialises a unit's gradient storage
  right before its backward and releases it after its reduce-scatter.
* The optimizer state (fp32 master, m, v) and the reduced gradient shard of every unit live
  in ONE per-dtype **arena**; the whole sharded AdamW update is one fused HIP kernel launch
  per dtype (ops.optim.adamw_flat), followed by async all-gathers of updated shards.
* Global-norm clipping: sum of squares of the local gradient shards, one all-reduce.
"""
from ..framework.flags import pa_flag  # noqa: E402
import math

import torch
import torch.distributed as dist

from ..core.tensor import Tensor, Parameter, _wrap, _unwrap
from .flat_buffer import FlatBuffer, ALIGN, register_grad_ready, run_pre_finish
from .. import ops

LEVELS = {'os': 1, 'os_g': 2, 'p_g_os': 3}


def _pg(group):
    return None if group is None else getattr(group, 'pg', group)


class _Unit:
    def __init__(self, engine, params, layer=None, persistent=True):
        self.engine = engine
        self.layer = layer
        self.persistent = persistent
        W = engine.world
        self.fb = FlatBuffer(params, pad_to_multiple=W)
        self.params = self.fb.params
        self.L = self.fb.numel // W
        self.dtype = self.fb.dtype
        self.gathered = True
        self.grad_live = True
        self.gather_work = None
        self.rs_work = None
        self.pending = sum(1 for p in self.params if p._t.requires_grad)
        # stage-3 parameters that are released after their layer's forward: consumers outside the
        # layer must not hold on to them (models/gpt.py defers a bias to the next block only when
        # this is False)
        releasable = engine.level == 3 and not persistent
        for p in self.params:
            p.__dict__['_releasable'] = releasable
        self.arena_off = None  # set by engine
        self.index = -1

    # ---- local shard views
    def shard(self, t):
        r = self.engine.rank
        return t[r * self.L:(r + 1) * self.L]

    # ---- parameter materialisation (stage 3)
    def free_params(self):
        if self.persistent or not self.gathered:
            return
        self.fb.data.untyped_storage().resize_(0)
        self.gathered = False

    def gather_async(self):
        if self.gathered or self.gather_work is not None:
            return
        st = self.fb.data.untyped_storage()
        st.resize_(self.fb.numel * self.fb.data.element_size())
        src = self.engine.pshard(self)
        if not self.engine.collectives:
            self.fb.data.copy_(src)
            self.gathered = True
            return
        self.gather_work = dist.all_gather_into_tensor(self.fb.data, src, group=self.engine.pg, async_op=True)

    def wait_gather(self):
        if self.gather_work is None and not self.gathered:
            self.gather_async()
        if self.gather_work is not None:
            self.gather_work.wait()
            self.gather_work = None
        self.gathered = True

    # ---- gradient storage (stage 3 releases it between steps)
    def alloc_grads(self):
        if self.grad_live:
            return
        st = self.fb.grad.untyped_storage()
        st.resize_(self.fb.numel * self.fb.grad.element_size())
        self.fb.grad.zero_()
        self.grad_live = True

    def free_grads(self):
        if self.grad_live and self.engine.release_grads:
            self.fb.grad.untyped_storage().resize_(0)
            self.grad_live = False


class _PreBackward(torch.autograd.Function):
    """Identity on a unit's outputs whose backward materialises the unit (params + grads)
    before autograd enters the unit's own backward."""

    @staticmethod
    def forward(ctx, unit_box, *xs):
        ctx.unit = unit_box[0]
        return xs if len(xs) > 1 else xs[0]

    @staticmethod
    def backward(ctx, *gs):
        u = ctx.unit
        u.engine._pre_backward(u)
        return (None,) + gs


class ShardingEngine:
    def __init__(self, model, level='p_g_os', group=None, bucket_mb=256, segment_size=2 ** 20,
                 release_grads=True, persistent_types=None, persistent_below=None, params=None, alias=None,
                 reduce_dtype=None, isolate=None, reshard_after_forward=None, offload=False):
        """model: the Layer to shard; or model=None with ``params`` (a parameter list) for stage 1/2
        (the hybrid-parallel sharding optimizer, which only sees its optimizer's parameters).

        alias: at world 1 the units alias the optimizer arenas (default); ``alias=False`` (or env
        PADDLE_AMD_SHARDING_ALIAS=0) runs the multi-rank code path on one rank — release, gather,
        re-materialise, shard copy — so it can be exercised on a single GPU.
        reduce_dtype: 'float32' reduce-scatters low-precision gradients in fp32 (fp32 main-grad
        communication, 2x the bytes) into an fp32 gradient arena; default: the parameter dtype.
        isolate: stage 1/2 only — ``isolate(p)`` returns a key or None; parameters with the same key
        form a unit of their own (pipeline-shared weights, whose shards must line up across the
        stages that hold a copy).
        reshard_after_forward (stage 3): release a unit's gathered parameters after its forward
        and all-gather them again for its backward (True), or keep them until the unit's gradient
        reduce-scatter (False: one all-gather per unit and step instead of two, the parameters of
        the whole model materialised at the forward/backward turn).  None: False on a GPU when the
        model's parameters take at most 1/16 of the device memory (288 GB HBM: e.g. GPT-3 1.3B's
        2.6 GB), else True; always True on the CPU.
        offload: the fp32 master weights and Adam moments of this rank's shard live in pinned host
        memory (12 bytes per shard element off the device); the step copies the gradient shard
        down, updates on the host runtime's worker pool (csrc/runtime pa_rt_adamw) and copies the
        16-bit parameter shard back (reference group_sharded_stage3.py:98-127 offload)."""
        self.model = model
        self.level = LEVELS[level] if isinstance(level, str) else int(level)
        if model is None and (params is None or self.level == 3):
            raise ValueError("ShardingEngine: stage 3 needs the model; stage 1/2 need model or params")
        self.group = group
        self.pg = _pg(group)
        self.world = dist.get_world_size(self.pg) if dist.is_initialized() else 1
        self.rank = dist.get_rank(self.pg) if dist.is_initialized() else 0
        # collectives: False only for a single rank with no forced collectives.  Forcing them
        # (PADDLE_AMD_FORCE_COLLECTIVES=1 with an initialised process group, e.g. a 1-rank RCCL
        # group) runs the real all-gather / reduce-scatter / all-reduce calls at world 1, so the
        # multi-GPU stream ordering is exercised on one GPU (the gradients then equal the world-1
        # result bit for bit: a 1-rank AVG / SUM is the identity).
        import os
        force = pa_flag('force_collectives') and dist.is_initialized()
        self.collectives = self.world > 1 or force
        # one rank: the "shard" is the whole buffer, so units alias the optimizer arenas and
        # nothing is ever released, gathered or copied (no degenerate collectives either)
        if alias is None:
            import os
            alias = pa_flag('sharding_alias')
        self.alias = not self.collectives and bool(alias)
        self.release_grads = release_grads and self.level == 3 and not self.alias
        self.reshard_after_forward = self._auto_reshard(model, params) if reshard_after_forward is None \
            else bool(reshard_after_forward)
        rd = str(reduce_dtype).replace('torch.', '').replace('paddle.', '') if reduce_dtype is not None else None
        if rd is None and self.level == 3 and self.world > 1:
            # stage 3 across ranks: an N-way bf16 / fp16 reduce-scatter rounds at every ring hop,
            # so 16-bit gradients are reduced in fp32 by default (reduce_dtype='param' opts out)
            rd = 'float32'
        elif rd == 'param':
            rd = None
        if rd not in (None, 'float32', 'bfloat16', 'float16'):
            raise ValueError(f"reduce_dtype must be float32 / bfloat16 / float16, got {reduce_dtype}")
        self.reduce_fp32 = rd == 'float32' and not self.alias
        self.offload = bool(offload)
        self._gather_works = []
        from ..nn.layer.common import Embedding
        self.persistent_types = tuple(persistent_types or (Embedding,))
        # units smaller than this stay materialised: gathering them saves nothing, and small
        # layers (norms, heads) are the ones parent code tends to use outside their own forward
        # (the reference likewise leaves parameters below segment_size unsliced, group_sharded_stage3.py)
        self.persistent_below = segment_size if persistent_below is None else persistent_below
        self._explicit_params = params
        self._broadcast_params()
        params = list(params) if params is not None else list(model.parameters())
        if self.level == 3:
            self.units = self._layer_units(model, segment_size)
        else:
            self.units = self._bucket_units(params, bucket_mb, isolate)
        for i, u in enumerate(self.units):
            u.index = i
        self._build_arenas()
        self._hooks = []
        self._install_grad_hooks()
        if self.level == 3:
            self._install_layer_hooks()
            for u in self.units:
                u.free_params()
                u.free_grads()
        self.hooks_off = False
        self._armed = False
        self._fwd_order = []
        self._recording = True
        self.grad_fresh = True
        # data-parallel replicas of the sharding group (hybrid parallelism): the gradient shard of
        # a unit is all-reduced over dp_pg as soon as it is final — on RCCL chained on the device
        # behind the unit's reduce-scatter (a side stream waits for it, the all-reduce is issued
        # from there), overlapping the rest of backward; dp_final is cleared by pipeline schedules
        # for every micro-batch but the last
        self.dp_pg = None
        self.dp_scale = None  # dp x sep groups: SUM scaled by 1/dp instead of the group average
        self.dp_final = True
        self.dp_defer = set()  # units whose dp all-reduce waits for step() (pipeline-shared weights)
        self._dp_works = []
        self._dp_done = set()
        self._dp_stream = None

    # ------------------------------------------------------------------ construction
    def _broadcast_params(self):
        if not self.collectives:
            return
        if self.model is None:  # replicas of every parameter start equal: broadcast from rank 0
            src = self.group.ranks[0] if self.group is not None and hasattr(self.group, 'ranks') else 0
            with torch.no_grad():
                for p in self._explicit_params:
                    dist.broadcast(p._t, src, group=self.pg)
            return
        from .data_parallel import sync_params_buffers
        sync_params_buffers(self.model, self.group)

    def _bucket_units(self, params, bucket_mb, isolate=None):
        units = []
        by_dt = {}
        own = {}
        for p in params:
            k = isolate(p) if isolate is not None else None
            if k is not None:
                own.setdefault((k, p._t.dtype), []).append(p)
            else:
                by_dt.setdefault(p._t.dtype, []).append(p)
        for _, ps in sorted(own.items(), key=lambda kv: str(kv[0])):
            units.append(_Unit(self, ps, None, True))
        cap = bucket_mb * 2 ** 20
        for dt, ps in by_dt.items():
            cur, size = [], 0
            for p in ps:
                cur.append(p)
                size += p._t.numel() * p._t.element_size()
                if size >= cap:
                    units.append(_Unit(self, cur, None, True))
                    cur, size = [], 0
            if cur:
                units.append(_Unit(self, cur, None, True))
        return units

    def _layer_units(self, model, segment_size):
        """Greedy top-down split: a layer whose subtree holds <= segment_size*64 elements becomes
        one unit (per dtype); bigger layers are descended into; a layer's *own* params are
        grouped into a unit for that layer."""
        limit = max(segment_size * 64, 1)
        units = []
        seen = set()

        def count(layer):
            return sum(p._t.numel() for p in layer.parameters() if id(p) not in seen)

        def make(layer, params, persistent):
            by_dt = {}
            for p in params:
                if id(p) in seen:
                    continue
                seen.add(id(p))
                by_dt.setdefault(p._t.dtype, []).append(p)
            for dt, ps in by_dt.items():
                small = sum(p._t.numel() for p in ps) < self.persistent_below
                units.append(_Unit(self, ps, layer, persistent or small or self.alias))

        def holds_persistent(layer):
            return any(isinstance(l, self.persistent_types) for l in layer.sublayers())

        def visit(layer):
            n = count(layer)
            if n == 0:
                return
            if isinstance(layer, self.persistent_types):
                make(layer, layer.parameters(), True)
                return
            children = [c for c in layer.children() if count(c) > 0]
            from ..nn.layer.container import LayerList, LayerDict
            container = isinstance(layer, (LayerList, LayerDict))  # never called: descend
            # a subtree holding an embedding is always descended into: the embedding must get its
            # own persistent unit (its weight is commonly tied to a head used outside the subtree)
            if (n <= limit and not container and not holds_persistent(layer)) or not children:
                make(layer, layer.parameters(), False)
                return
            own = [p for p in layer._parameters.values() if p is not None]
            if own:
                make(layer, own, True)
            for c in children:
                visit(c)

        visit(model)
        return units

    def _build_arenas(self):
        self.arenas = {}
        for u in self.units:
            a = self.arenas.setdefault(u.dtype, {'units': [], 'size': 0})
            u.arena_off = a['size']
            a['size'] += u.L
            a['units'].append(u)
        for dt, a in self.arenas.items():
            n = a['size']
            dev = a['units'][0].fb.data.device
            a['param'] = torch.empty(n, dtype=dt, device=dev)
            gdt = torch.float32 if self.reduce_fp32 else dt
            a['grad'] = torch.zeros(n, dtype=gdt, device=dev)
            for u in a['units']:
                if self.alias:
                    u.fb.alias_into(a['param'][u.arena_off:u.arena_off + u.L],
                                    a['grad'][u.arena_off:u.arena_off + u.L])
                else:
                    a['param'][u.arena_off:u.arena_off + u.L].copy_(u.shard(u.fb.data))
            if self.offload:  # optimizer state in (pinned) host memory, staging buffers for the step
                pin = dev.type == 'cuda'
                a['master'] = torch.empty(n, dtype=torch.float32, pin_memory=pin)
                a['master'].copy_(a['param'].float())
                a['m'] = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
                a['v'] = torch.zeros(n, dtype=torch.float32, pin_memory=pin)
                a['grad_host'] = torch.empty(n, dtype=a['grad'].dtype, pin_memory=pin)
                a['param_host'] = torch.empty(n, dtype=dt, pin_memory=pin)
            else:
                a['master'] = a['param'].float().clone() if dt != torch.float32 else a['param']
                a['m'] = torch.zeros(n, dtype=torch.float32, device=dev)
                a['v'] = torch.zeros(n, dtype=torch.float32, device=dev)
            a['b1p'] = None

    def _auto_reshard(self, model, params):
        ps = list(params) if params is not None else (list(model.parameters()) if model is not None else [])
        if not ps or not ps[0]._t.is_cuda:
            return True
        nbytes = sum(p._t.numel() * p._t.element_size() for p in ps)
        total = torch.cuda.get_device_properties(ps[0]._t.device).total_memory
        return nbytes * 16 > total

    def pshard(self, u):
        return self.arenas[u.dtype]['param'][u.arena_off:u.arena_off + u.L]

    def gshard(self, u):
        return self.arenas[u.dtype]['grad'][u.arena_off:u.arena_off + u.L]

    # ------------------------------------------------------------------ hooks
    def _install_grad_hooks(self):
        for u in self.units:
            for p in u.params:
                if p._t.requires_grad:
                    self._hooks.append(register_grad_ready(p, self._grad_hook(u)))

    def _grad_hook(self, u):
        def hook():
            if not self._armed:
                self._armed = True
                torch.autograd.Variable._execution_engine.queue_callback(self._finish_backward)
            u.pending -= 1
            if u.pending == 0:
                self._reduce_scatter(u)
        return hook

    def _install_layer_hooks(self):
        for u in self.units:
            if u.persistent or u.layer is None:
                continue
            layer = u.layer
            layer.register_forward_pre_hook(self._fwd_pre(u))
            layer.register_forward_post_hook(self._fwd_post(u))
        # persistent units of stage 3 are gathered at the start of every forward
        self.model.register_forward_pre_hook(self._root_pre)

    def _root_pre(self, layer, inputs):
        if self.hooks_off:
            return None
        for u in self.units:
            if u.persistent or u.layer is None:
                u.wait_gather()
                if torch.is_grad_enabled():
                    u.alloc_grads()
        return None

    def _fwd_pre(self, u):
        def hook(layer, inputs):
            if self.hooks_off:
                return None
            if self._recording and torch.is_grad_enabled():
                self._fwd_order.append(u)
            u.wait_gather()
            if torch.is_grad_enabled():
                u.alloc_grads()
            # prefetch the next unit in forward order
            nxt = self._next_unit(u, +1)
            if nxt is not None:
                nxt.gather_async()
            return None
        return hook

    def _fwd_post(self, u):
        def hook(layer, inputs, outputs):
            if self.hooks_off:  # static recording (dist.to_static): the replay gathers up front
                return outputs
            if torch.is_grad_enabled():
                outs = outputs if isinstance(outputs, tuple) else (outputs,)
                idx = [i for i, o in enumerate(outs) if isinstance(o, Tensor) and o._t.requires_grad]
                if idx:
                    ts = [outs[i]._t for i in idx]
                    res = _PreBackward.apply([u], *ts)
                    res = res if isinstance(res, tuple) else (res,)
                    new = list(outs)
                    for i, r in zip(idx, res):
                        new[i] = _wrap(r)
                    outputs = tuple(new) if isinstance(outputs, tuple) else new[0]
                if self.reshard_after_forward:
                    u.free_params()  # else kept until its gradient reduce-scatter (no backward re-gather)
            else:
                u.free_params()
            return outputs
        return hook

    def _next_unit(self, u, direction):
        order = self._fwd_order
        if not order or self._recording:
            return None
        try:
            i = self._order_index[id(u)]
        except (AttributeError, KeyError):
            return None
        j = i + direction
        return order[j] if 0 <= j < len(order) else None

    def _pre_backward(self, u):
        u.wait_gather()
        u.alloc_grads()
        prv = self._next_unit(u, -1)
        if prv is not None:
            prv.gather_async()

    # ------------------------------------------------------------------ gradient reduction
    def _reduce_scatter(self, u):
        if self.alias:
            u.rs_work = None  # gradients already live in the arena
            return
        if not self.collectives:
            u.rs_work = None
            self._accumulate_shard(u, u.shard(u.fb.grad))
            return
        gs = self.gshard(u)
        out = gs if self.grad_fresh else torch.empty(u.L, dtype=gs.dtype, device=gs.device)
        u._rs_out = out
        src = u.fb.grad if u.fb.grad.dtype == out.dtype else u.fb.grad.to(out.dtype)  # fp32 main-grad reduce
        op = dist.ReduceOp.AVG if dist.get_backend(self.pg) == 'nccl' else dist.ReduceOp.SUM
        u.rs_work = dist.reduce_scatter_tensor(out, src, op, group=self.pg, async_op=True)
        if self.dp_pg is not None and self.dp_final and self.grad_fresh and dist.get_backend(self.pg) == 'nccl':
            self._launch_dp(u)  # out IS the shard: chain the dp all-reduce behind the reduce-scatter
        if self.level == 3:
            u.free_params()

    def _launch_dp(self, u):
        """Async all-reduce (average) of unit u's gradient shard over the data-parallel group."""
        if self.dp_pg is None or u.index in self._dp_done:
            return
        if u.index in self.dp_defer and not getattr(self, '_dp_flush', False):
            return
        gs = self.gshard(u)
        nccl = dist.get_backend(self.dp_pg) == 'nccl'
        op = dist.ReduceOp.AVG if nccl and self.dp_scale is None else dist.ReduceOp.SUM
        if nccl and gs.is_cuda and u.rs_work is not None:
            if self._dp_stream is None:
                self._dp_stream = torch.cuda.Stream(device=gs.device)
            side = self._dp_stream
            side.wait_stream(torch.cuda.current_stream(gs.device))
            with torch.cuda.stream(side):
                u.rs_work.wait()  # device-side: the side stream waits for the reduce-scatter
                w = dist.all_reduce(gs, op, group=self.dp_pg, async_op=True)
        else:
            w = dist.all_reduce(gs, op, group=self.dp_pg, async_op=True)
        self._dp_works.append((gs, w, nccl))
        self._dp_done.add(u.index)

    def finish_dp_sync(self, dp_nranks):
        """Launch the dp all-reduce of every unit not yet launched, then wait for all of them."""
        if self.dp_pg is None:
            return
        self._dp_flush = True
        try:
            for u in self.units:
                self._launch_dp(u)
        finally:
            self._dp_flush = False
        for gs, w, nccl in self._dp_works:
            w.wait()
            if self.dp_scale is not None:
                gs.mul_(self.dp_scale)
            elif not nccl:
                gs.div_(dp_nranks)
        self._dp_works = []
        self._dp_done = set()

    def _accumulate_shard(self, u, src):
        dst = self.gshard(u)
        if self.grad_fresh:
            if src.data_ptr() != dst.data_ptr():
                dst.copy_(src)
        else:
            dst.add_(src.to(dst.dtype))

    def _finish_backward(self):
        run_pre_finish()  # deferred gradient kernels (ops.linear grouped weight gradients) land first
        for u in self.units:
            if u.pending > 0 and u.rs_work is None:
                if not u.grad_live:
                    u.alloc_grads()
                self._reduce_scatter(u)
        for u in self.units:
            if u.rs_work is not None:
                u.rs_work.wait()
                u.rs_work = None
                if dist.get_backend(self.pg) != 'nccl':
                    u._rs_out.div_(self.world)
                if not self.grad_fresh:
                    self.gshard(u).add_(u._rs_out)
            u.pending = sum(1 for p in u.params if p._t.requires_grad)
            if u.grad_live and not self.release_grads and not self.alias:
                u.fb.grad.zero_()
            u.free_grads()
            u.free_params()
            if self.dp_pg is not None and self.dp_final:
                self._launch_dp(u)  # shard final (accumulated / CPU path): its dp all-reduce goes now
        self.grad_fresh = False
        if self._recording and self._fwd_order:
            self._recording = False
            self._order_index = {id(x): i for i, x in enumerate(self._fwd_order)}
        self._armed = False

    def zero_grad(self):
        for a in self.arenas.values():
            a['grad'].zero_()
        self.grad_fresh = True
        self._dp_works = []
        self._dp_done = set()

    # ------------------------------------------------------------------ after the update
    def gather_params_after_step(self):
        """Re-materialise updated parameters.  Stage 1/2 with a model: one ASYNC all-gather per
        unit, waited for by the model's forward pre-hook (the gathers overlap whatever the host
        does between step() and the next forward: data loading, logging, LR scheduling);
        without a model (hybrid-parallel sharding optimizer) the gathers are waited for here."""
        for u in self.units:
            if u.persistent or self.level < 3:
                if not self.collectives:
                    if not u.gathered:  # released persistent unit (alias off): plain re-materialise
                        u.wait_gather()
                    elif u.fb.data.data_ptr() != self.pshard(u).data_ptr():
                        u.fb.data[:u.L].copy_(self.pshard(u))
                    continue
                w = dist.all_gather_into_tensor(u.fb.data, self.pshard(u), group=self.pg, async_op=True)
                self._gather_works.append(w)
            else:
                # stage-3 non-persistent units are gathered lazily by their forward pre-hook; one
                # still holding (or prefetching) pre-step weights — e.g. gathered by a grad-enabled
                # forward after the last backward — is released so the next forward re-gathers
                if u.gather_work is not None:
                    u.gather_work.wait()
                    u.gather_work = None
                    u.gathered = True
                u.free_params()
        if self.model is None or self.level == 3:
            self.wait_param_gathers()
        elif not getattr(self, '_gather_hook_installed', False):
            # every sublayer waits before it runs or hands out its state dict, so a read through
            # the original (inner) layer never sees a half-written parameter
            for layer in self.model.sublayers(include_self=True):
                layer.register_forward_pre_hook(lambda layer, inputs: self.wait_param_gathers())
                layer.register_state_dict_hook(self._state_dict_wait)
            self._gather_hook_installed = True

    def _state_dict_wait(self, dest):
        self.wait_param_gathers()
        return None

    def wait_param_gathers(self):
        ws, self._gather_works = self._gather_works, []
        for w in ws:
            w.wait()
        return None


class ShardedOptimizer:
    """Wraps a paddle optimizer; updates only the local shard.  Adam/AdamW: one fused HIP AdamW
    launch per dtype arena (fp32 master + moments); SGD / Momentum (L2 regularisation, Nesterov):
    a flat elementwise update of the arena, the velocity sharded like the moments.

    Reference: GroupShardedOptimizerStage2 / the stage-3 _OptimizerWrapper."""

    SUPPORTED = ('AdamW', 'Adam', 'SGD', 'Momentum')

    def __init__(self, optimizer, engine):
        self._inner = optimizer
        self.engine = engine
        self._step = 0
        name = type(optimizer).__name__
        if name not in self.SUPPORTED:
            raise NotImplementedError(f"group-sharded training supports {self.SUPPORTED}, got {name}")
        self._kind = name
        self._decoupled = name == 'AdamW'
        self._coeff_runs = {}
        for dt, a in engine.arenas.items():
            self._coeff_runs[dt] = self._runs(a)

    def _coeff(self, p):
        opt = self._inner
        if self._kind in ('SGD', 'Momentum'):  # L2 regularisation coefficient (added to the gradient)
            from ..regularizer import L2Decay
            reg = getattr(p, 'regularizer', None) or opt.regularization
            if reg is None:
                return 0.0
            if isinstance(reg, (int, float)):
                return float(reg)
            if isinstance(reg, L2Decay):
                return float(reg._coeff)
            raise NotImplementedError(f"group-sharded {self._kind} supports L2Decay regularisation only, got "
                                      f"{type(reg).__name__}")
        if not self._decoupled:
            return 0.0
        f = getattr(opt, '_apply_decay_param_fun', None)
        if f is not None and not f(p.name):
            return 0.0
        return float(opt._coeff)

    def _runs(self, arena, key=None):
        """(arena_lo, arena_hi, value) runs of equal ``key(param)`` (default: weight decay)
        covering [0, arena size)."""
        key = key or self._coeff
        segs = []
        r = self.engine.rank
        for u in arena['units']:
            lo_s, hi_s = r * u.L, (r + 1) * u.L
            for p, o in zip(u.fb.params, u.fb.offsets):
                a, b = max(o, lo_s), min(o + p._t.numel(), hi_s)
                if a < b:
                    segs.append((u.arena_off + (a - lo_s), u.arena_off + (b - lo_s), key(p)))
        segs.sort()
        runs = []
        for a, b, c in segs:
            if runs and runs[-1][2] == c:
                runs[-1][1] = b
            else:
                if runs:
                    runs[-1][1] = a  # padding between params rides with the previous run
                runs.append([a, b, c])
        if not runs:
            return [[0, arena['size'], 0.0]]
        runs[0][0] = 0
        runs[-1][1] = arena['size']
        return runs

    # ---- paddle optimizer surface
    def get_lr(self):
        return self._inner.get_lr()

    def set_lr(self, v):
        self._inner.set_lr(v)

    @property
    def _learning_rate(self):
        return self._inner._learning_rate

    def _clip_scale(self):
        clip = self._inner._grad_clip
        if clip is None:
            return None
        from ..nn.clip import ClipGradByGlobalNorm
        if not isinstance(clip, ClipGradByGlobalNorm):
            return None
        sq = None
        for a in self.engine.arenas.values():
            g = a['grad']
            s = ops.optim.sumsq(g) if ops.use_hip(g) else g.float().pow(2).sum()
            sq = s if sq is None else sq + s
        if clip._extra_sq_norm_fn is not None:
            sq = clip._extra_sq_norm_fn(sq)
        if self.engine.collectives:
            dist.all_reduce(sq, group=self.engine.pg)
        norm = sq.sqrt()
        return torch.clamp(clip.clip_norm / torch.clamp(norm, min=clip.clip_norm), max=1.0)

    @torch.no_grad()
    def _step_sgd_momentum(self, lr, scale, offload=False):
        opt = self._inner
        mom = self._kind == 'Momentum'
        mu = float(getattr(opt, '_momentum', 0.0))
        nesterov = bool(getattr(opt, '_use_nesterov', False))
        rescale = float(getattr(opt, '_rescale', 1.0))
        for dt, a in self.engine.arenas.items():
            if offload:  # host master / velocity, the gradient shard already copied down
                lowp, grad = a['param_host'], a['grad_host']
            else:
                lowp, grad = (a['param'] if dt != torch.float32 else None), a['grad']
            for lo, hi, coeff in self._coeff_runs[dt]:
                if hi <= lo:
                    continue
                master = a['master'][lo:hi]
                g = grad[lo:hi].float()
                if scale is not None:
                    g = g * scale
                if mom and rescale != 1.0:
                    g = g * rescale  # reference momentum: rescale_grad * g + coeff * param
                if coeff:
                    g = g + coeff * master
                if mom:
                    v = a['m'][lo:hi]
                    v.mul_(mu).add_(g)
                    upd = g + mu * v if nesterov else v
                else:
                    upd = g
                master.sub_(upd * lr if torch.is_tensor(lr) else lr * upd)
                if lowp is not None:
                    lowp[lo:hi].copy_(master.to(dt))

    _DTC = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}

    @torch.no_grad()
    def _step_offload(self):
        """The update with the optimizer state in host memory: per arena one async D2H of the
        gradient shard, the native host AdamW (or the SGD / Momentum rule) over the worker pool,
        one H2D of the updated parameter shard."""
        from .. import _runtime as R
        opt = self._inner
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("sharding offload cannot run inside a captured step graph")
        self._step += 1
        lr = float(opt.get_lr())
        scale = self._clip_scale()
        gs = 1.0 if scale is None else float(scale)
        for a in self.engine.arenas.values():
            a['grad_host'].copy_(a['grad'], non_blocking=True)
        if any(a['grad'].is_cuda for a in self.engine.arenas.values()):
            torch.cuda.current_stream().synchronize()
        if self._kind in ('SGD', 'Momentum'):
            self._step_sgd_momentum(lr, None if scale is None else gs, offload=True)
        else:
            b1, b2, eps = opt._beta1, opt._beta2, opt._epsilon
            b1p, b2p = b1 ** self._step, b2 ** self._step
            L = R.lib()
            for dt, a in self.engine.arenas.items():
                gh, ph = a['grad_host'], a['param_host']
                for lo, hi, coeff in self._coeff_runs[dt]:
                    if hi <= lo:
                        continue
                    es = a['master'].element_size()
                    rc = L.pa_rt_adamw(a['master'].data_ptr() + lo * es, gh.data_ptr() + lo * gh.element_size(),
                                       self._DTC[gh.dtype], a['m'].data_ptr() + lo * es, a['v'].data_ptr() + lo * es,
                                       ph.data_ptr() + lo * ph.element_size(), self._DTC[ph.dtype], hi - lo, lr,
                                       b1, b2, eps, float(coeff), b1p, b2p, gs)
                    if rc:
                        raise RuntimeError(f"pa_rt_adamw failed ({rc})")
        for a in self.engine.arenas.values():
            a['param'].copy_(a['param_host'], non_blocking=True)
        self.engine.gather_params_after_step()
        opt._global_step += 1

    @torch.no_grad()
    def step(self):
        if self.engine.offload:
            return self._step_offload()
        opt = self._inner
        self._step += 1
        lr = opt.get_lr()
        lr_dev = self._graph_lr()
        scale = self._clip_scale()
        if self._kind in ('SGD', 'Momentum'):
            self._step_sgd_momentum(lr if lr_dev is None else lr_dev, scale)
            self.engine.gather_params_after_step()
            opt._global_step += 1
            return
        b1, b2, eps = opt._beta1, opt._beta2, opt._epsilon
        b1p, b2p = b1 ** self._step, b2 ** self._step
        # device copy of the powers for steps captured into a hipGraph (the host values would be
        # frozen at capture); created on an eager step, advanced on the device after each update
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        pows = getattr(self, '_pows', None)
        if pows is None and not capturing and any(ops.use_hip(a['master']) for a in self.engine.arenas.values()):
            dev = next(iter(self.engine.arenas.values()))['master'].device
            pows = self._pows = torch.tensor([b1p, b2p], dtype=torch.float32, device=dev)
            self._betas = torch.tensor([b1, b2], dtype=torch.float32, device=dev)
        for dt, a in self.engine.arenas.items():
            g = a['grad']
            if scale is not None and not ops.use_hip(g):
                g.mul_(scale.to(g.dtype))
            lowp = a['param'] if dt != torch.float32 else None
            for lo, hi, coeff in self._coeff_runs[dt]:
                if hi <= lo:
                    continue
                if ops.use_hip(a['master']):
                    ops.optim.adamw_flat(a['master'][lo:hi], g[lo:hi], a['m'][lo:hi], a['v'][lo:hi],
                                         None if lowp is None else lowp[lo:hi], lr, b1, b2, eps, coeff, b1p, b2p,
                                         lr_tensor=lr_dev, grad_scale=scale, pows=pows if capturing else None)
                else:
                    _adamw_ref(a['master'][lo:hi], g[lo:hi], a['m'][lo:hi], a['v'][lo:hi],
                               None if lowp is None else lowp[lo:hi], lr, b1, b2, eps, coeff, b1p, b2p)
        if pows is not None:
            pows.mul_(self._betas)
        self.engine.gather_params_after_step()
        opt._global_step += 1

    def _graph_lr(self):
        """Device fp32 [1] learning rate while a TrainStepGraph captures this step: refilled from
        the inner optimizer's get_lr() before every replay; the host step counters advance after
        each replay (device/cuda/graphs.py on_replay).  None otherwise (host value).  Allocated on
        an eager step, not from the capture's private pool (a block an earlier temporary of the
        captured step used would be overwritten by the replay after the pre-replay fill)."""
        if not torch.cuda.is_available():
            return None
        lr_dev = getattr(self, '_lr_dev', None)
        if not torch.cuda.is_current_stream_capturing():
            if lr_dev is None and self.engine.arenas:
                dev = next(iter(self.engine.arenas.values()))['master'].device
                if dev.type == 'cuda':
                    self._lr_dev = torch.zeros(1, dtype=torch.float32, device=dev)
            return None
        if lr_dev is None:
            return None
        from ..device.cuda.graphs import on_replay
        opt = self._inner

        def post():
            self._step += 1
            opt._global_step += 1
        return lr_dev if on_replay(pre=lambda: lr_dev.fill_(opt.get_lr()), post=post) else None

    def clear_grad(self, set_to_zero=True):
        self.engine.zero_grad()

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def state_dict(self):
        self.engine.wait_param_gathers()
        sd = {}
        for dt, a in self.engine.arenas.items():
            key = str(dt).replace('torch.', '')
            sd[f'shard_master_{key}'] = _wrap(a['master'])
            sd[f'shard_moment1_{key}'] = _wrap(a['m'])
            sd[f'shard_moment2_{key}'] = _wrap(a['v'])
        sd['@step@'] = self._step
        if hasattr(self._inner._learning_rate, 'state_dict'):
            sd['LR_Scheduler'] = self._inner._learning_rate.state_dict()
        return sd

    def set_state_dict(self, sd):
        for dt, a in self.engine.arenas.items():
            key = str(dt).replace('torch.', '')
            for nm, buf in (('master', a['master']), ('moment1', a['m']), ('moment2', a['v'])):
                v = sd.get(f'shard_{nm}_{key}')
                if v is not None:
                    buf.copy_(_unwrap(v).to(buf.device))
            if dt != torch.float32 or self.engine.offload:
                a['param'].copy_(a['master'].to(dt))
        self._step = int(sd.get('@step@', self._step))
        pows = getattr(self, '_pows', None)
        if pows is not None and self._kind not in ('SGD', 'Momentum'):
            # in place: a TrainStepGraph captured before the load keeps reading this tensor (powers
            # of the NEXT update, step + 1)
            b1, b2 = self._inner._beta1, self._inner._beta2
            nxt = self._step + 1
            pows.copy_(torch.tensor([b1 ** nxt, b2 ** nxt], dtype=torch.float32))
        if 'LR_Scheduler' in sd and hasattr(self._inner._learning_rate, 'set_state_dict'):
            self._inner._learning_rate.set_state_dict(sd['LR_Scheduler'])
        self.engine.gather_params_after_step()

    def __getattr__(self, name):
        return getattr(self._inner, name)


def _adamw_ref(p, g, m, v, lowp, lr, b1, b2, eps, wd, b1p, b2p):
    gg = g.float()
    p.mul_(1 - lr * wd)
    m.mul_(b1).add_(gg, alpha=1 - b1)
    v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    bc2 = math.sqrt(1 - b2p)
    p.sub_(lr * bc2 / (1 - b1p) * m / (v.sqrt() + eps * bc2))
    if lowp is not None:
        lowp.copy_(p.to(lowp.dtype))


class GroupShardedModel:
    """The wrapped model returned by group_sharded_parallel (a Layer proxy)."""

    def __new__(cls, layer, engine):
        from ..nn.layer.layers import Layer

        class _GS(Layer):
            def __init__(self):
                super().__init__()
                self._layers = layer
                self.__dict__['_engine'] = engine

            def forward(self, *a, **k):
                return self._layers(*a, **k)

            def state_dict(self, *a, **k):
                return gathered_state_dict(self._layers, engine)

            def set_state_dict(self, sd, use_structured_name=True):
                return self._layers.set_state_dict(sd, use_structured_name)

            def get_all_parameters(self, convert2cpu=False):
                engine.wait_param_gathers()
                for u in engine.units:
                    u.wait_gather()
                return self._layers.parameters()

        _GS.__name__ = 'GroupShardedStage%d' % engine.level
        return _GS()


def gathered_state_dict(layer, engine):
    """Full (unsharded) state dict: gathers any released unit, copies, releases again."""
    out = {}
    engine.wait_param_gathers()
    released = [u for u in engine.units if not u.gathered]
    for u in released:
        u.wait_gather()
    for k, v in layer.state_dict().items():
        out[k] = _wrap(v._t.detach().clone())
    for u in released:
        u.free_params()
    return out
