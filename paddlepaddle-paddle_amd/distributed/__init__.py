"""paddle.distributed (reference: python/paddle/distributed/__init__.py)."""
from .communication import (ReduceOp, Group, all_reduce, all_gather, all_gather_object, broadcast,  # noqa: F401
                            broadcast_object_list, reduce, reduce_scatter, scatter, scatter_object_list, gather,
                            alltoall, alltoall_single, send, recv, isend, irecv, batch_isend_irecv, P2POp, barrier,
                            wait, new_group, get_group, destroy_process_group, is_initialized, is_available,
                            get_backend, split, stream)
from .parallel import ParallelEnv, init_parallel_env, get_rank, get_world_size, spawn  # noqa: F401
from ..parallel.data_parallel import DataParallel  # noqa: F401
from . import sharding  # noqa: F401
from . import watchdog  # noqa: F401


def gloo_init_parallel_env(rank_id, rank_num, server_endpoint):
    """CPU-side gloo group (reference: parallel.py gloo_init_parallel_env)."""
    import torch.distributed as _d
    host, port = server_endpoint.split(':')
    if not _d.is_initialized():
        _d.init_process_group('gloo', init_method=f"tcp://{host}:{port}", rank=rank_id, world_size=rank_num)


def gloo_barrier():
    import torch.distributed as _d
    if _d.is_initialized():
        _d.barrier()


def gloo_release():
    import torch.distributed as _d
    if _d.is_initialized() and _d.get_backend() == 'gloo':
        _d.destroy_process_group()


from .fleet.dataset import (InMemoryDataset, QueueDataset, CountFilterEntry, ProbabilityEntry,  # noqa: E402,F401
                            ShowClickEntry)
import importlib as _il


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3
    SEGMENT_PARALLEL = 4


_LAZY = {'fleet': '.fleet', 'launch': '.launch', 'auto_parallel': '.auto_parallel', 'checkpoint': '.checkpoint',
         'utils': '.utils', 'io': '.io', 'rpc': '.rpc', 'passes': '.passes'}
_AUTO = ('ProcessMesh', 'DistAttr', 'shard_tensor', 'dtensor_from_fn', 'reshard', 'shard_layer', 'shard_dataloader',
         'ReduceType', 'Placement', 'Shard', 'Replicate', 'Partial', 'shard_optimizer', 'shard_scaler',
         'ShardingStage1', 'ShardingStage2', 'ShardingStage3', 'to_static', 'Strategy', 'DistModel',
         'unshard_dtensor', 'set_mesh', 'get_mesh')


def __getattr__(name):
    if name in _LAZY:
        m = _il.import_module(_LAZY[name], __name__)
        globals()[name] = m
        return m
    if name in _AUTO:
        m = _il.import_module('.auto_parallel', __name__)
        return getattr(m, name)
    if name in ('save_state_dict', 'load_state_dict'):
        m = _il.import_module('.checkpoint', __name__)
        return getattr(m, name)
    raise AttributeError(f"module 'paddle.distributed' has no attribute '{name}'")
