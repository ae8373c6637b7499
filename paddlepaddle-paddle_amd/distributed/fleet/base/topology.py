"""Hybrid-parallel topology (reference: python/paddle/distributed/fleet/base/topology.py).

Axes ["data", "pipe", "sharding", "sep", "model"], rank = row-major coordinate (model axis
innermost, so tensor-parallel peers are adjacent ranks — on an 8×MI355X node every pair is
one xGMI hop, and adjacent ranks share a switch-free link).  One RCCL communicator is created
per (axis, coordinate-of-the-other-axes) group, exactly once, on every rank.
"""
import collections
import itertools
from functools import reduce

import torch.distributed as dist

from ...communication import new_group, Group


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3
    SEGMENT_PARALLEL = 4


class CommunicateTopology:
    def __init__(self, hybrid_group_names=("data", "pipe", "sharding", "sep", "model"), dims=(1, 1, 1, 1, 1)):
        self._parallel_names = list(hybrid_group_names)
        self._dims = list(dims)
        self.coordinate = collections.namedtuple('Coordinate', self._parallel_names)
        self._world_size = reduce(lambda a, b: a * b, self._dims, 1)
        coords = [self.coordinate(*c) for c in itertools.product(*[range(d) for d in self._dims])]
        self._coord2rank = {c: i for i, c in enumerate(coords)}
        self._rank2coord = {i: c for c, i in self._coord2rank.items()}

    def get_hybrid_group_names(self):
        return self._parallel_names

    def get_dim(self, axis_name):
        return self._dims[self._parallel_names.index(axis_name)]

    get_dim_size = get_dim

    def world_size(self):
        return self._world_size

    def get_rank(self, **kw):
        return self._coord2rank[self.coordinate(**kw)]

    def get_coord(self, rank):
        return self._rank2coord[rank]

    def get_axis_list(self, axis_name, index):
        ax = self._parallel_names.index(axis_name)
        return sorted(r for c, r in self._coord2rank.items() if c[ax] == index)

    def get_comm_list(self, axis_name):
        others = [n for n in self._parallel_names if n != axis_name]
        out = []
        for x in itertools.product(*[range(self.get_dim(n)) for n in others]):
            kc = dict(zip(others, x))
            grp = []
            for i in range(self.get_dim(axis_name)):
                kc[axis_name] = i
                grp.append(self._coord2rank[self.coordinate(**kc)])
            out.append(grp)
        return out

    def get_fused_ranks(self, fused_axis):
        non = [n for n in self._parallel_names if n not in fused_axis]
        out = []
        for x in itertools.product(*[range(self.get_dim(n)) for n in non]):
            kc = dict(zip(non, x))
            ranks = []
            for y in itertools.product(*[range(self.get_dim(n)) for n in fused_axis]):
                kc.update(dict(zip(fused_axis, y)))
                ranks.append(self._coord2rank[self.coordinate(**kc)])
            out.append(sorted(ranks))
        return out

    def get_rank_from_stage(self, global_rank, **kwargs):
        c = self.get_coord(global_rank)._replace(**kwargs)._asdict()
        return self.get_rank(**c)


class HybridCommunicateGroup:
    def __init__(self, topology):
        self._topo = topology
        self.nranks = dist.get_world_size() if dist.is_initialized() else 1
        self.global_rank = dist.get_rank() if dist.is_initialized() else 0
        assert self.nranks == topology.world_size(), \
            f"topology world size {topology.world_size()} != launched ranks {self.nranks}"
        self._dp_degree = topology.get_dim('data')
        self._pp_degree = topology.get_dim('pipe')
        self._sharding_degree = topology.get_dim('sharding')
        self._sep_degree = topology.get_dim('sep')
        self._mp_degree = topology.get_dim('model')
        self.stage_id = topology.get_coord(self.global_rank).pipe
        self._groups = {}
        for axis in topology.get_hybrid_group_names():
            mine = None
            for ranks in topology.get_comm_list(axis):
                g = self._mk(ranks)
                if self.global_rank in ranks:
                    mine = g
            self._groups[axis] = mine
        # fused groups used by checks / hybrid clip
        self._check_group = self._mk_fused(['data', 'pipe', 'sharding', 'sep', 'model'])
        self._dp_sep_group = self._mk_fused(['data', 'sep']) if self._sep_degree > 1 else self._groups['data']
        self._pp_mp_group = self._mk_fused(['pipe', 'model'])
        self._set_p2p()

    def _mk(self, ranks):
        if len(ranks) == 1 or not dist.is_initialized():
            return Group(0 if self.global_rank in ranks else -1, -1, ranks, None)
        return new_group(ranks)

    def _mk_fused(self, axes):
        mine = None
        for ranks in self._topo.get_fused_ranks(axes):
            g = self._mk(ranks)
            if self.global_rank in ranks:
                mine = g
        return mine

    def _set_p2p(self):
        pp = self._pp_degree
        coord = self._topo.get_coord(self.global_rank)
        self.next_rank = self._topo.get_rank(**coord._replace(pipe=(coord.pipe + 1) % pp)._asdict())
        self.prev_rank = self._topo.get_rank(**coord._replace(pipe=(coord.pipe - 1) % pp)._asdict())

    # ---- reference accessors
    def get_parallel_mode(self):
        # precedence pp -> mp -> sep -> sharding -> dp (reference topology.py:290-320)
        if self._pp_degree > 1:
            return ParallelMode.PIPELINE_PARALLEL
        if self._mp_degree > 1:
            return ParallelMode.TENSOR_PARALLEL  # may coexist with sep, sharding, dp
        if self._sep_degree > 1:
            return ParallelMode.SEGMENT_PARALLEL  # may coexist with sharding, dp
        if self._sharding_degree > 1:
            return ParallelMode.SHARDING_PARALLEL
        return ParallelMode.DATA_PARALLEL

    def topology(self):
        return self._topo

    def get_global_rank(self):
        return self.global_rank

    def _axis_rank(self, axis):
        return getattr(self._topo.get_coord(self.global_rank), axis)

    def get_data_parallel_rank(self):
        return self._axis_rank('data')

    def get_data_parallel_world_size(self):
        return self._dp_degree

    def get_data_parallel_group(self):
        return self._groups['data']

    def get_data_parallel_group_src_rank(self):
        return self._groups['data'].ranks[0]

    def get_model_parallel_rank(self):
        return self._axis_rank('model')

    def get_model_parallel_world_size(self):
        return self._mp_degree

    def get_model_parallel_group(self):
        return self._groups['model']

    def get_model_parallel_group_src_rank(self):
        return self._groups['model'].ranks[0]

    def get_stage_id(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self._pp_degree

    def get_pipe_parallel_group(self):
        return self._groups['pipe']

    def get_sharding_parallel_rank(self):
        return self._axis_rank('sharding')

    def get_sharding_parallel_world_size(self):
        return self._sharding_degree

    def get_sharding_parallel_group(self):
        return self._groups['sharding']

    def get_sharding_parallel_group_src_rank(self):
        return self._groups['sharding'].ranks[0]

    def get_sep_parallel_rank(self):
        return self._axis_rank('sep')

    def get_sep_parallel_world_size(self):
        return self._sep_degree

    def get_sep_parallel_group(self):
        return self._groups['sep']

    def get_sep_parallel_group_src_rank(self):
        return self._groups['sep'].ranks[0]

    def get_check_parallel_group(self, sharding=False):
        return self._check_group

    def get_dp_sep_parallel_group(self):
        return self._dp_sep_group

    def get_pp_mp_parallel_group(self):
        return self._pp_mp_group

    def get_rank_from_stage(self, stage_id, **kwargs):
        return self._topo.get_rank_from_stage(self.global_rank, pipe=stage_id, **kwargs)

    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self._pp_degree - 1
