"""paddle.incubate.distributed.fleet (reference: python/paddle/incubate/distributed/fleet/__init__.py):
the recompute entry points re-exported from the fleet recompute package."""
from ....distributed.fleet.recompute import recompute_hybrid, recompute_sequential  # noqa: F401

__all__ = ["recompute_sequential", "recompute_hybrid"]
