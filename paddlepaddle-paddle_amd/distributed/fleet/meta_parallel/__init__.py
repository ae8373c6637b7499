"""paddle.distributed.fleet.meta_parallel (reference: .../fleet/meta_parallel/__init__.py)."""
from .pipeline import (LayerDesc, SharedLayerDesc, SegmentLayers, PipelineLayer, PipelineParallel,  # noqa: F401
                       PipelineParallelWithInterleave, PipelineParallelWithInterleaveFthenB)
from . import sharding  # noqa: F401,E402
from ..layers.mpu import (VocabParallelEmbedding, ColumnParallelLinear, RowParallelLinear,  # noqa: F401
                          ParallelCrossEntropy, get_rng_state_tracker, model_parallel_random_seed)
from ....nn.layer.layers import Layer as _Layer


class TensorParallel(_Layer):
    """Wraps a model built from mpu layers: broadcasts replicated params over mp / dp groups."""

    def __init__(self, layers, hcg, strategy=None):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        from ..utils.hybrid_parallel_util import broadcast_mp_parameters, broadcast_dp_parameters
        # replicated (non-distributed) params must agree across the mp group
        import torch.distributed as dist
        import torch
        g = hcg.get_model_parallel_group()
        if g is not None and g.nranks > 1:
            with torch.no_grad():
                for p in layers.parameters():
                    if not getattr(p, 'is_distributed', False):
                        dist.broadcast(p._t, hcg.get_model_parallel_group_src_rank(), group=g.pg)
        broadcast_dp_parameters(layers, hcg)

    def forward(self, *a, **k):
        return self._layers(*a, **k)

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layers.set_state_dict(*a, **k)


class ShardingParallel(TensorParallel):
    pass


class SegmentParallel(TensorParallel):
    pass
