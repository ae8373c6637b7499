"""Reference auto_parallel/interface.py: the legacy shard_tensor / shard_op entry points."""
from .api import shard_tensor, reshard, ProcessMesh  # noqa: F401


def shard_op(op, process_mesh=None, in_shard_specs=None, out_shard_specs=None, **kwargs):
    """Annotates a callable with its process mesh; the SPMD rules propagate its placements, so the
    callable itself is returned (reference interface.py shard_op)."""
    return op
