"""HybridParallelOptimizer lives with fleet (distributed/fleet/__init__.py); re-exported here at the
reference's import path (fleet/meta_optimizers/dygraph_optimizer/hybrid_parallel_optimizer.py)."""
from ....fleet import HybridParallelOptimizer  # noqa: F401
