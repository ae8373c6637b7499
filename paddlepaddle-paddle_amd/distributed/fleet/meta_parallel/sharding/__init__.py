"""paddle.distributed.fleet.meta_parallel.sharding — the module path of the reference's group-sharded
classes (reference: python/paddle/distributed/fleet/meta_parallel/sharding/).  The engine is
parallel/sharding.py (flat per-unit buffers, reduce-scatter / all-gather over RCCL); these are the
reference's constructor surfaces over it."""
from .group_sharded_optimizer_stage2 import GroupShardedOptimizerStage2  # noqa: F401
from .group_sharded_stage2 import GroupShardedStage2  # noqa: F401
from .group_sharded_stage3 import GroupShardedStage3  # noqa: F401
from .group_sharded_utils import GroupShardedScaler, GroupShardedClipGrad  # noqa: F401
from .group_sharded_storage import ParamStorage, GradStorage, InternalStorage  # noqa: F401
