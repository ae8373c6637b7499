"""paddle.distributed.fleet (reference: python/paddle/distributed/fleet/fleet.py:100 Fleet,
base/distributed_strategy.py, model.py:32 distributed_model, optimizer.py distributed_optimizer).

``fleet.init(is_collective=True, strategy=s)`` builds the hybrid topology from
``s.hybrid_configs`` (dp/mp/pp/sharding/sep degrees) and one RCCL communicator per axis group;
``distributed_model`` wraps the model for the active parallel mode (DataParallel,
TensorParallel, PipelineParallel, or group-sharded); ``distributed_optimizer`` wraps the
optimizer so that gradient clipping sees the global norm across model-parallel shards and
sharding partitions.
"""
import copy

import torch
import torch.distributed as dist

from .base.topology import CommunicateTopology, HybridCommunicateGroup, ParallelMode  # noqa: F401
from . import layers, meta_parallel, utils  # noqa: F401
from .recompute import recompute, recompute_sequential, recompute_hybrid  # noqa: F401
from .meta_parallel import (LayerDesc, SharedLayerDesc, PipelineLayer, ColumnParallelLinear,  # noqa: F401
                            RowParallelLinear, VocabParallelEmbedding, ParallelCrossEntropy, get_rng_state_tracker)


class DistributedStrategy:
    """Subset of the reference's protobuf-backed strategy, as plain attributes."""

    def __init__(self):
        self.hybrid_configs = {'dp_degree': -1, 'mp_degree': 1, 'pp_degree': 1, 'sharding_degree': 1,
                               'sep_degree': 1, 'order': ['dp', 'pp', 'sharding', 'sep', 'mp'],
                               'mp_configs': {}, 'pp_configs': {}}
        self.pipeline_configs = {'accumulate_steps': 1, 'micro_batch_size': 1, 'schedule_mode': '1F1B'}
        self.sharding = False
        self.sharding_configs = {'sharding_degree': 1, 'stage': 1, 'segment_broadcast_MB': 32}
        self.amp = False
        self.amp_configs = {'init_loss_scaling': 32768.0, 'use_pure_fp16': False, 'use_pure_bf16': False,
                            'custom_white_list': [], 'custom_black_list': []}
        self.recompute = False
        self.recompute_configs = {'checkpoints': [], 'enable_offload': False}
        self.gradient_merge = False
        self.gradient_merge_configs = {'k_steps': 1, 'avg': True}
        self.tensor_parallel = False
        self.tensor_parallel_configs = {'tensor_parallel_degree': 1}
        self.pipeline = False
        self.fuse_all_reduce_ops = True
        self.fuse_grad_size_in_MB = 64
        self.find_unused_parameters = False
        self.without_graph_optimization = False
        self.heter_ccl_mode = False
        self.lamb = False
        self.lars = False
        self.dgc = False
        self.localsgd = False
        self.a_sync = False
        self.nccl_comm_num = 1

    def __setattr__(self, k, v):
        if k.endswith('_configs') and k in self.__dict__ and isinstance(v, dict):
            d = dict(self.__dict__[k])
            d.update(v)
            object.__setattr__(self, k, d)
        else:
            object.__setattr__(self, k, v)

    def __repr__(self):
        return f"DistributedStrategy(hybrid_configs={self.hybrid_configs})"


class _Fleet:
    def __init__(self):
        self._hcg = None
        self._strategy = None
        self._is_collective = True
        self._inited = False
        self._ps = None

    def init(self, role_maker=None, is_collective=True, strategy=None, log_level="INFO"):
        if role_maker is not None and getattr(role_maker, '_is_collective', None) is False:
            is_collective = False
        if not is_collective:  # parameter-server mode (distributed/ps): no collective world
            from ..ps import PSRuntime
            self._strategy = strategy or DistributedStrategy()
            self._is_collective = False
            self._ps = PSRuntime()
            self._inited = True
            return None
        from ..parallel import init_parallel_env
        init_parallel_env()
        self._strategy = strategy or DistributedStrategy()
        self._is_collective = is_collective
        world = dist.get_world_size() if dist.is_initialized() else 1
        hc = self._strategy.hybrid_configs
        mp, pp = int(hc.get('mp_degree', 1)), int(hc.get('pp_degree', 1))
        sh, sep = int(hc.get('sharding_degree', 1)), int(hc.get('sep_degree', 1))
        dp = int(hc.get('dp_degree', -1))
        if dp == -1:
            dp = max(world // (mp * pp * sh * sep), 1)
        topo = CommunicateTopology(["data", "pipe", "sharding", "sep", "model"], [dp, pp, sh, sep, mp])
        self._hcg = HybridCommunicateGroup(topo)
        self._topology = topo
        self._inited = True
        if mp > 1:
            from .layers.mpu.random import model_parallel_random_seed
            model_parallel_random_seed(2024)
        return None

    def get_hybrid_communicate_group(self):
        return self._hcg

    def worker_index(self):
        if not self._is_collective:
            return 0 if self._ps.role.is_server else self._ps.role.index
        return dist.get_rank() if dist.is_initialized() else 0

    def worker_num(self):
        if not self._is_collective:
            return self._ps.role.num_trainers
        return dist.get_world_size() if dist.is_initialized() else 1

    def is_first_worker(self):
        return self.is_worker() and self.worker_index() == 0

    def is_worker(self):
        return self._is_collective or not self._ps.role.is_server

    def is_server(self):
        return (not self._is_collective) and self._ps.role.is_server

    def server_num(self):
        return 0 if self._is_collective else self._ps.role.num_servers

    def server_index(self):
        return self._ps.role.index if self.is_server() else 0

    def server_endpoints(self, to_string=False):
        eps = [] if self._is_collective else list(self._ps.role.servers)
        return ','.join(eps) if to_string else eps

    # ---- parameter-server lifecycle (reference fleet.py:893-1063)
    def init_server(self, *args, **kwargs):
        self._ps.init_server()

    def run_server(self):
        self._ps.run_server()

    def init_worker(self, scopes=None):
        self._ps.init_worker()

    def stop_worker(self):
        self._ps.stop_worker()

    def barrier_worker(self):
        if dist.is_initialized():
            dist.barrier()

    def worker_endpoints(self, to_string=False):
        import os
        eps = os.environ.get('PADDLE_TRAINER_ENDPOINTS', '').split(',')
        return ','.join(eps) if to_string else eps

    def distributed_model(self, model):
        hcg = self._hcg
        if hcg is None:
            return model
        mode = hcg.get_parallel_mode()
        if mode == ParallelMode.PIPELINE_PARALLEL:
            if getattr(model, 'get_num_virtual_stages', lambda: 1)() > 1:
                cfg = getattr(self._strategy, 'pipeline_configs', {}) or {}
                acc, pp = int(cfg.get('accumulate_steps', 1)), hcg.get_pipe_parallel_world_size()
                if pp <= acc < 2 * pp:  # the reference's choice (fleet/model.py:168)
                    return meta_parallel.PipelineParallelWithInterleaveFthenB(model, hcg, self._strategy)
                if acc < pp:
                    raise ValueError(f"The accumulate_steps({acc}) should be greater than or equal to pp_degree({pp})")
                return meta_parallel.PipelineParallelWithInterleave(model, hcg, self._strategy)
            return meta_parallel.PipelineParallel(model, hcg, self._strategy)
        if mode == ParallelMode.TENSOR_PARALLEL:
            return meta_parallel.TensorParallel(model, hcg, self._strategy)
        if mode == ParallelMode.SEGMENT_PARALLEL:
            return meta_parallel.SegmentParallel(model, hcg, self._strategy)
        if mode == ParallelMode.SHARDING_PARALLEL:
            return model  # wrapped together with the optimizer by distributed_optimizer / group_sharded_parallel
        from ...parallel.data_parallel import DataParallel
        if hcg.get_data_parallel_world_size() > 1:
            return DataParallel(model, comm_buffer_size=self._strategy.fuse_grad_size_in_MB,
                                find_unused_parameters=self._strategy.find_unused_parameters,
                                group=hcg.get_data_parallel_group())
        return model

    def distributed_optimizer(self, optimizer, strategy=None):
        if strategy is not None:
            self._strategy = strategy
        if not self._is_collective:
            from ..ps import PSOptimizer
            return PSOptimizer(optimizer, self._ps, self._strategy)
        from ...framework import in_dynamic_mode
        if not in_dynamic_mode():  # static Program + Executor: collective data parallelism
            return StaticCollectiveOptimizer(optimizer, self._hcg, self._strategy or DistributedStrategy())
        hcg = self._hcg
        if hcg is None:
            return optimizer
        if hcg.get_sharding_parallel_world_size() > 1:
            # the sharding axis: reduce-scattered gradients, sharded optimizer state, parameter
            # all-gather after the step (plus the dp all-reduce of the shards)
            from .meta_optimizers.dygraph_optimizer import DygraphShardingOptimizer
            return DygraphShardingOptimizer(optimizer, hcg, self._strategy)
        return HybridParallelOptimizer(optimizer, hcg, self._strategy)

    def distributed_scaler(self, scaler):
        """reference fleet/scaler.py: the found-inf flag is max-reduced over every rank of the
        hybrid topology (a shard or pipeline stage that overflowed makes all ranks skip the step)."""
        def sync(found):
            import torch
            dev = found.device if isinstance(found, torch.Tensor) else (
                torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() and
                dist.get_backend() == 'nccl' else torch.device('cpu'))
            t = found.detach().float().reshape(1).clone() if isinstance(found, torch.Tensor) else \
                torch.tensor([1.0 if found else 0.0], device=dev)
            if dist.is_initialized() and dist.get_world_size() > 1:
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return bool(t.item() > 0)
        scaler._sync_found_inf = sync
        return scaler

    def save_persistables(self, executor, dirname, main_program=None):
        from ..io import save_persistables
        save_persistables(executor, dirname, main_program)

    @property
    def util(self):
        return utils


class StaticCollectiveOptimizer:
    """``fleet.distributed_optimizer`` in static mode (reference: fleet/meta_optimizers/
    raw_program_optimizer.py + amp / gradient_merge meta optimizers, which rewrite the program
    with c_broadcast of the parameters in the startup program and c_allreduce_sum of every
    gradient).  ``minimize`` records the backward/update node and installs its step policy
    (static/minimize.py): strategy.amp -> static AMP (amp_configs), strategy.gradient_merge ->
    k-step merge, data-parallel gradient averaging over the data (x sharding) ranks in
    ``fuse_grad_size_in_MB`` buckets.  Parameters are broadcast from the group's first rank when
    the program is built, so every rank starts from the same weights.  Tensor parallelism: the
    fleet mpu layers (ColumnParallelLinear / RowParallelLinear / VocabParallelEmbedding /
    ParallelCrossEntropy) record their c_identity / c_allreduce / c_split / c_concat collectives as
    program nodes, which run the eager RCCL ops (and their backward) when the Executor replays the
    program.  Pipeline parallelism: ops recorded under ``static.device_guard('gpu:N')`` form stage
    N; each rank runs its stage's section with ``pipeline_configs`` accumulate_steps micro-batches
    (FThenB / 1F1B) and send/recv of the boundary activations and gradients (static/pipeline.py)."""

    def __init__(self, optimizer, hcg, strategy):
        self._inner_opt = optimizer
        self._hcg = hcg
        self._strategy = strategy
        self._policy = None

    def __getattr__(self, name):
        return getattr(self.__dict__['_inner_opt'], name)

    def _dp_group(self):
        hcg = self._hcg
        if hcg is None:
            return None
        # tensor parallel: the mpu layers record their collectives as program nodes (mp_ops
        # _static_value); gradients are averaged over the data-parallel group only
        if hcg.get_sharding_parallel_world_size() > 1:
            # static sharding trains like data parallelism over data x sharding ranks (the reference's
            # static sharding pass shards the optimizer state; the update is the same)
            from ..communication import new_group
            return new_group(list(range(dist.get_world_size())))
        g = hcg.get_data_parallel_group()
        return g if g is not None and g.nranks > 1 else None

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        from ...static.program import _static_minimize
        from ...static.minimize import step_policy
        from ...static.program import default_main_program
        s = self._strategy
        opt = self._inner_opt
        if s.amp:
            from ...static import amp as samp
            c = s.amp_configs
            pure = bool(c.get('use_pure_fp16') or c.get('use_pure_bf16'))
            dtype = 'bfloat16' if (c.get('use_pure_bf16') or c.get('use_bf16') or c.get('dtype') == 'bfloat16') \
                else 'float16'
            lists = samp.AutoMixedPrecisionLists(custom_white_list=c.get('custom_white_list') or None,
                                                 custom_black_list=c.get('custom_black_list') or None, dtype=dtype)
            opt = samp.decorate(opt, amp_lists=lists, level='O2' if pure else 'O1', dtype=dtype,
                                init_loss_scaling=c.get('init_loss_scaling', 32768.0),
                                use_dynamic_loss_scaling=c.get('use_dynamic_loss_scaling', None),
                                incr_every_n_steps=c.get('incr_every_n_steps', 1000),
                                decr_every_n_nan_or_inf=c.get('decr_every_n_nan_or_inf', 2),
                                incr_ratio=c.get('incr_ratio', 2.0), decr_ratio=c.get('decr_ratio', 0.8))
            res = opt.minimize(loss, startup_program, parameter_list, no_grad_set)
        else:
            res = _static_minimize(opt, loss, parameter_list, no_grad_set)
        prog = default_main_program()
        pol = step_policy(prog)
        if s.gradient_merge:
            pol.k_steps = max(1, int(s.gradient_merge_configs.get('k_steps', 1)))
            pol.avg = bool(s.gradient_merge_configs.get('avg', True))
        pol.dp_group = self._dp_group()
        pol.fuse_grad_size_in_MB = s.fuse_grad_size_in_MB
        hcg = self._hcg
        if hcg is not None and hcg.get_pipe_parallel_world_size() > 1:
            # static pipeline: the program runs split by device_guard stage (static/pipeline.py)
            from ...static.pipeline import PipelineConfig
            pc = dict(getattr(s, 'pipeline_configs', None) or {})
            grp = hcg.get_pipe_parallel_group()
            st_id, S = hcg.get_stage_id(), hcg.get_pipe_parallel_world_size()
            ranks = list(grp.ranks)
            mode = str(pc.get('schedule_mode', '1F1B'))
            vpp = int(pc.get('vpp_degree', 1) or 1) if mode.upper() == 'VPP' else 1
            grad_grp = None
            if vpp > 1:  # interleaved stages: gradients on a communicator of their own
                for rk in hcg.topology().get_comm_list('pipe'):  # collective: every rank, same order
                    g = hcg._mk(rk)
                    if hcg.global_rank in rk:
                        grad_grp = g
            pol.pipeline = PipelineConfig(st_id, S, pc.get('accumulate_steps', 1), grp,
                                          ranks[st_id - 1] if st_id > 0 else None,
                                          ranks[st_id + 1] if st_id < S - 1 else None,
                                          mode, vpp=vpp, grad_group=grad_grp)
        if pol.dp_group is not None:
            _broadcast_params(pol._params(), pol.dp_group)
        self._policy = pol
        return res


def _broadcast_params(params, group):
    """Parameters from the group's first rank (the reference's startup-program c_broadcast)."""
    pg = getattr(group, 'pg', None)
    src = group.ranks[0] if getattr(group, 'ranks', None) else 0
    with torch.no_grad():
        for p in params:
            dist.broadcast(p._t.data, src=src, group=pg)


class HybridParallelOptimizer:
    """reference: fleet/meta_optimizers/dygraph_optimizer/hybrid_parallel_optimizer.py.

    Makes ClipGradByGlobalNorm global across the hybrid topology: the squared norm of
    tensor-parallel (distributed) parameters is summed over the mp group, replicated ones are
    counted once; pipeline stages sum over the pp group."""

    def __init__(self, optimizer, hcg, strategy):
        self._inner_opt = optimizer
        self._hcg = hcg
        self._strategy = strategy
        clip = getattr(optimizer, '_grad_clip', None)
        from ...nn.clip import ClipGradByGlobalNorm
        if isinstance(clip, ClipGradByGlobalNorm):
            clip._extra_sq_norm_fn = self._global_sq

    def _global_sq(self, sq):
        mp = self._hcg.get_model_parallel_group()
        pp = self._hcg.get_pipe_parallel_group()
        if mp is not None and mp.nranks > 1:
            # every param on an mp rank is either a shard (distinct) or a replica (identical on all
            # ranks): sum shards' norms over mp, count replicas once (they were counted on every rank)
            dist_sq = torch.zeros_like(sq)
            rep_sq = torch.zeros_like(sq)
            for p in self._inner_opt._parameter_list:
                g = p._t.grad
                if g is None:
                    continue
                s = g.float().pow(2).sum()
                if getattr(p, 'is_distributed', False):
                    dist_sq = dist_sq + s
                else:
                    rep_sq = rep_sq + s
            dist.all_reduce(dist_sq, group=mp.pg)
            sq = dist_sq + rep_sq
        if pp is not None and pp.nranks > 1:
            # a pipeline-shared weight's copies on later stages are not counted again
            dup = [p for p in self._inner_opt._parameter_list
                   if (p.__dict__.get('_pp_shared') or (None, False))[1] and p._t.grad is not None]
            if dup:
                def _sq(ps):
                    if not ps:
                        return torch.zeros_like(sq)
                    return torch.stack([p._t.grad.float().pow(2).sum() for p in ps]).sum().to(sq.dtype)
                dup_dist = [p for p in dup if getattr(p, 'is_distributed', False)]
                dup_rep = [p for p in dup if not getattr(p, 'is_distributed', False)]
                d_dist = _sq(dup_dist)
                if mp is not None and mp.nranks > 1:
                    # tensor-parallel shards of a shared weight were summed over mp above; the
                    # same ranks hold the same stage, so this collective is uniform over mp
                    dist.all_reduce(d_dist, group=mp.pg)
                sq = sq - d_dist - _sq(dup_rep)
            sq = sq.clone()
            dist.all_reduce(sq, group=pp.pg)
        return sq

    def step(self):
        # tensor-parallel (and sep) models are not wrapped in DataParallel: their gradients are
        # all-reduced over the dp group here (reference hybrid_parallel_optimizer.py: step ->
        # fused_allreduce_gradients).  Pipeline schedules sync dp themselves before stepping.
        # Parameters of a model wrapped by TensorParallel / SegmentParallel were reduced during
        # backward (hook-driven buckets on the dp x sep group); anything else goes here, bucketed.
        mode = self._hcg.get_parallel_mode()
        from .utils.hybrid_parallel_util import dp_sep_group_and_scale, fused_allreduce_gradients
        grp = dp_sep_group_and_scale(self._hcg)[0]
        if mode in (ParallelMode.TENSOR_PARALLEL, ParallelMode.SEGMENT_PARALLEL) and grp is not None \
                and grp.nranks > 1:
            fused_allreduce_gradients(list(self._inner_opt._parameter_list), self._hcg)
        self._inner_opt.step()

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def clear_grad(self, set_to_zero=True):
        self._inner_opt.clear_grad(set_to_zero)

    def __getattr__(self, name):
        return getattr(self._inner_opt, name)


fleet = _Fleet()
init = fleet.init
get_hybrid_communicate_group = fleet.get_hybrid_communicate_group
distributed_model = fleet.distributed_model
distributed_optimizer = fleet.distributed_optimizer
distributed_scaler = fleet.distributed_scaler
worker_index = fleet.worker_index
worker_num = fleet.worker_num
is_first_worker = fleet.is_first_worker
barrier_worker = fleet.barrier_worker
worker_endpoints = fleet.worker_endpoints
is_server = fleet.is_server
is_worker = fleet.is_worker
init_server = fleet.init_server
run_server = fleet.run_server
init_worker = fleet.init_worker
stop_worker = fleet.stop_worker
server_num = fleet.server_num
server_index = fleet.server_index
server_endpoints = fleet.server_endpoints


def _inited():
    return fleet._inited


class UserDefinedRoleMaker:
    def __init__(self, *a, **k):
        pass


class PaddleCloudRoleMaker(UserDefinedRoleMaker):
    """Roles from the PADDLE_* / TRAINING_ROLE environment (reference role_maker.py)."""

    def __init__(self, is_collective=False, **kwargs):
        self._is_collective = is_collective


class Role:
    WORKER = 1
    SERVER = 2


class UtilBase:
    """fleet.util (reference: python/paddle/distributed/fleet/base/util_factory.py): collective helpers
    over the worker group plus file sharding for data-parallel input lists."""

    def _t(self, x):
        import numpy as np
        import torch
        return torch.as_tensor(np.asarray(x))

    def all_reduce(self, input, mode="sum", comm_world="worker"):
        import torch
        import torch.distributed as tdist
        t = self._t(input).clone()
        if tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1:
            op = {'sum': tdist.ReduceOp.SUM, 'max': tdist.ReduceOp.MAX, 'min': tdist.ReduceOp.MIN}[mode]
            tdist.all_reduce(t, op=op)
        return t.numpy()

    def barrier(self, comm_world="worker"):
        import torch.distributed as tdist
        if tdist.is_available() and tdist.is_initialized():
            tdist.barrier()

    def all_gather(self, input, comm_world="worker"):
        import torch.distributed as tdist
        if tdist.is_available() and tdist.is_initialized() and tdist.get_world_size() > 1:
            out = [None] * tdist.get_world_size()
            tdist.all_gather_object(out, input)
            return out
        return [input]

    def get_file_shard(self, files):
        """This worker's contiguous share of ``files`` (earlier workers take one extra file when
        the count does not divide)."""
        if not isinstance(files, list):
            raise TypeError("files should be a list of file paths")
        n, i = fleet.worker_num(), fleet.worker_index()
        base, extra = divmod(len(files), n)
        start = i * base + min(i, extra)
        return files[start:start + base + (1 if i < extra else 0)]

    def print_on_rank(self, message, rank_id):
        if fleet.worker_index() == rank_id:
            print(message)


util = UtilBase()
Fleet = _Fleet  # the class behind the module-level ``fleet`` singleton (reference fleet/fleet.py)
from . import data_generator  # noqa: E402,F401
from . import auto  # noqa: E402,F401
from .data_generator import MultiSlotDataGenerator, MultiSlotStringDataGenerator  # noqa: E402,F401


_ = copy
