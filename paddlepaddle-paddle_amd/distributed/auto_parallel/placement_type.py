"""Reference auto_parallel/placement_type.py: the placement classes (defined in api.py)."""
from .api import Placement, Shard, Replicate, Partial, ReduceType  # noqa: F401
