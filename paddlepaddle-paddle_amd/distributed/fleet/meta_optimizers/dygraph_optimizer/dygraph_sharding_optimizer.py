"""The sharding axis of Fleet hybrid parallelism (reference:
python/paddle/distributed/fleet/meta_optimizers/dygraph_optimizer/dygraph_sharding_optimizer.py:44
DygraphShardingOptimizer; reduce_gradients:316, _sharding_sync_parameters:358).

Returned by ``fleet.distributed_optimizer`` whenever ``sharding_degree > 1``.  The sharding group
is a data-parallel axis whose replicas split the optimizer state:

* the optimizer's parameters are re-homed into flat buffers cut into units
  (parallel/sharding.ShardingEngine, stage 2 'os_g'): rank s of the sharding group owns slice s
  of every unit; the moment a unit's gradients are complete (post-accumulate hooks, so this
  overlaps the rest of backward, and repeats per pipeline micro-batch) its flat gradient is
  reduce-scattered (AVG) over the sharding group into the rank's shard;
* ``step``: the gradient shards are all-reduced over the data-parallel group (1/sharding of the
  bytes a plain DP all-reduce would move), the global norm for ClipGradByGlobalNorm is summed
  shard -> sharding group -> model-parallel group (distributed parameters summed, replicated ones
  once) -> pipeline group, the local shard is updated (fused AdamW, or SGD / Momentum) with fp32
  master weights held only for the shard, and the updated shards are all-gathered over the
  sharding group.

Every rank therefore holds 1/sharding_degree of the fp32 master weights and moments.
"""
import torch
import torch.distributed as dist

from .....parallel.sharding import ShardingEngine, ShardedOptimizer


def _shared_key(p):
    """Pipeline-shared (SharedLayerDesc) parameters carry (key, duplicate) — see PipelineLayer."""
    s = p.__dict__.get('_pp_shared')
    return s[0] if s else None


class DygraphShardingOptimizer(ShardedOptimizer):
    _syncs_dp = True  # the pipeline schedule must not all-reduce gradients over dp itself

    def __init__(self, optimizer, hcg, strategy=None, level='os_g'):
        self._hcg = hcg
        params = [p for p in optimizer._parameter_list]
        sh = hcg.get_sharding_parallel_group()
        engine = ShardingEngine(None, level=level, group=sh, params=params,
                                bucket_mb=int(getattr(strategy, 'fuse_grad_size_in_MB', 256) or 256)
                                if strategy is not None else 256, isolate=_shared_key)
        super().__init__(optimizer, engine)
        self._dist_runs = {dt: self._runs(a, key=lambda p: 1.0 if getattr(p, 'is_distributed', False) else 0.0)
                           for dt, a in engine.arenas.items()}
        from ...utils.hybrid_parallel_util import dp_sep_group_and_scale
        dp, dp_scale = dp_sep_group_and_scale(hcg)
        if dp is not None and dp.nranks > 1:
            # overlapped gradient-shard all-reduce over the dp replicas (dp x sep when the sequence
            # is split too: summed over sep, averaged over dp)
            engine.dp_pg = dp.pg
            if hcg.get_sep_parallel_world_size() > 1:
                engine.dp_scale = dp_scale
            # pipeline-shared weights are summed over their stages after backward: their dp
            # all-reduce waits for step() (two in-place collectives must not race on one shard)
            engine.dp_defer = {u.index for u in engine.units if any(_shared_key(p) is not None for p in u.params)}

    # ---- gradient synchronisation across the data-parallel replicas of every sharding group
    def _dp_sync(self):
        """Gradient shards averaged over the data-parallel replicas.  The all-reduce of each unit
        was launched during backward the moment its shard was final (ShardingEngine._launch_dp:
        chained behind the unit's reduce-scatter on the device, overlapping the remaining backward);
        here the few not yet launched go out and every one is waited for."""
        from ...utils.hybrid_parallel_util import dp_sep_group_and_scale
        dp = dp_sep_group_and_scale(self._hcg)[0]
        if dp is None or dp.nranks <= 1:
            return
        self.engine.finish_dp_sync(self._hcg.get_data_parallel_world_size())

    def _shared_units(self):
        for u in self.engine.units:
            k = {_shared_key(p) for p in u.params}
            if len(k) == 1 and None not in k:
                yield next(iter(k)), u

    @torch.no_grad()
    def _sync_shared_grads(self, comm):
        """Sum the gradient shards of each pipeline-shared weight over the stages holding it (its
        unit has the same parameters, hence the same slicing, on all of them)."""
        for k, u in self._shared_units():
            g = comm.get(k)
            if g is not None:
                dist.all_reduce(self.engine.gshard(u), group=g.pg)

    def _clip_scale(self):
        clip = self._inner._grad_clip
        from .....nn.clip import ClipGradByGlobalNorm
        if clip is None or not isinstance(clip, ClipGradByGlobalNorm):
            return None
        # [distributed, replicated] squared norms of this rank's shard
        sq = None
        for dt, a in self.engine.arenas.items():
            g = a['grad']
            for lo, hi, isd in self._dist_runs[dt]:
                if hi <= lo:
                    continue
                s = g[lo:hi].float().pow(2).sum()
                v = torch.stack([s * isd, s * (1.0 - isd)])
                sq = v if sq is None else sq + v
        if sq is None:
            return None
        for _, u in self._shared_units():  # a shared weight's copies on later stages: not counted again
            if u.params[0].__dict__['_pp_shared'][1]:
                s = self.engine.gshard(u).float().pow(2).sum()
                isd = 1.0 if getattr(u.params[0], 'is_distributed', False) else 0.0
                sq = sq - torch.stack([s * isd, s * (1.0 - isd)])
        if self.engine.collectives:
            dist.all_reduce(sq, group=self.engine.pg)  # shards -> this stage's full local norm
        mp = self._hcg.get_model_parallel_group()
        if mp is not None and mp.nranks > 1:
            d = sq[0:1].clone()
            dist.all_reduce(d, group=mp.pg)  # tensor-parallel shards are distinct: sum them
            total = d[0] + sq[1]             # replicated parameters: counted once
        else:
            total = sq[0] + sq[1]
        pp = self._hcg.get_pipe_parallel_group()
        if pp is not None and pp.nranks > 1:
            total = total.reshape(1).clone()
            dist.all_reduce(total, group=pp.pg)
            total = total[0]
        norm = total.sqrt()
        return torch.clamp(clip.clip_norm / torch.clamp(norm, min=clip.clip_norm), max=1.0)

    @torch.no_grad()
    def step(self):
        self._dp_sync()
        super().step()

    def reduce_gradients(self, parameter_list=None, hcg=None):
        """Reference API: gradients are already reduce-scattered by the backward hooks; this
        flushes any unit whose gradients never completed (unused parameters)."""
        self.engine._finish_backward()

    def _sharding_sync_parameters(self):
        self.engine.gather_params_after_step()

    @property
    def _parameter_list(self):
        return self._inner._parameter_list
