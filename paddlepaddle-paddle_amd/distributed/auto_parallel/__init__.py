"""paddle.distributed.auto_parallel (reference: python/paddle/distributed/auto_parallel/): process
meshes, placements, dist tensors and reshard (api.py), the sharded optimizer / scaler /
dataloader wrappers, dist.to_static's DistModel and the static Engine (static/engine.py)."""
from .api import (  # noqa: F401
    Placement, Shard, Replicate, Partial, ReduceType, ProcessMesh, DistAttr, shard_tensor, dtensor_from_fn,
    reshard, unshard_dtensor, shard_layer, ShardingStage1, ShardingStage2, ShardingStage3, shard_optimizer,
    shard_scaler, shard_dataloader, Strategy, DistModel, to_static, is_dist_tensor, set_mesh, get_mesh,
    _dist_meta, _attach, _local_slice, _ensure_mesh_groups, _subgroup, _ShardOptimizer,
)
from .static.engine import Engine  # noqa: F401
from . import api, static  # noqa: F401
