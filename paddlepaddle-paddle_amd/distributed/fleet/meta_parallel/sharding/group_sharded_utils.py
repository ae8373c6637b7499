"""group_sharded_utils (reference: meta_parallel/sharding/group_sharded_utils.py): the scaler and
gradient-clip adapters.  The engine's sharded optimizer already reduces the global gradient norm
across the sharding group (one all-reduce of the shards' sums of squares) and a GradScaler's
unscale / inf check runs on the gradients it is given, so both adapters are thin."""
from .....nn.clip import ClipGradByGlobalNorm


def GroupShardedScaler(scaler):
    """Reference wraps the scaler's unscale to sum found-inf over the sharding group; the sharded
    optimizer's gradients are reduce-scattered before the scaler sees them, so any inf on one rank
    is on the shard every rank reduces from — the scaler is returned unchanged."""
    return scaler


class GroupShardedClipGrad:
    """Global-norm clip over sharded gradients (reference: GroupShardedClipGrad:48); the sharded
    optimizer applies ClipGradByGlobalNorm itself, this keeps the constructor surface."""

    def __init__(self, clip, device, group):
        self._clip = clip
        self._device = device
        self._group = group

    def __call__(self, params_grads):
        return self._clip(params_grads) if isinstance(self._clip, ClipGradByGlobalNorm) else params_grads

    def __getattr__(self, item):
        return getattr(self.__dict__['_clip'], item)
