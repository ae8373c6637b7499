"""paddle.distributed.fleet.meta_optimizers (reference: python/paddle/distributed/fleet/meta_optimizers)."""
from .dygraph_optimizer import DygraphShardingOptimizer, HybridParallelOptimizer  # noqa: F401
