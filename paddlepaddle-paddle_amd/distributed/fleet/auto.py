"""``paddle.distributed.fleet.auto`` (reference: python/paddle/distributed/fleet/auto.py re-exporting
the auto-parallel static API): Engine, Strategy, ProcessMesh, shard_tensor, shard_op."""
from ..auto_parallel import Engine, Strategy, ProcessMesh, shard_tensor, reshard, Shard, Replicate, Partial  # noqa: F401


def shard_op(op, process_mesh=None, in_shard_specs=None, out_shard_specs=None, **kwargs):
    """Annotate an op's placement (reference static annotation); eager SPMD propagation decides the
    placements of its outputs, so the op is returned unchanged."""
    return op
