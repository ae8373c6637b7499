"""paddle.distributed.auto_parallel.static (reference: python/paddle/distributed/auto_parallel/
static/): the static-graph auto-parallel Engine."""
from .engine import Engine  # noqa: F401
from .planner import RuleBasedPlanner, Planner, Plan  # noqa: F401

__all__ = ['Engine', 'RuleBasedPlanner', 'Planner', 'Plan']
