"""paddle.distributed.fleet.meta_parallel (reference: .../fleet/meta_parallel/__init__.py,
tensor_parallel.py, segment_parallel.py, sharding_parallel.py)."""
from .pipeline import (LayerDesc, SharedLayerDesc, SegmentLayers, PipelineLayer, PipelineParallel,  # noqa: F401
                       PipelineParallelWithInterleave, PipelineParallelWithInterleaveFthenB)
from . import sharding  # noqa: F401,E402
from ..layers.mpu import (VocabParallelEmbedding, ColumnParallelLinear, RowParallelLinear,  # noqa: F401
                          ParallelCrossEntropy, get_rng_state_tracker, model_parallel_random_seed)
from ....nn.layer.layers import Layer as _Layer


class MetaParallelBase(_Layer):
    """Wraps the user's model for one hybrid-parallel mode (reference meta_parallel_base.py):
    ``_prepare_for_model`` synchronises the replicated parameters over the axes whose ranks must
    hold the same weights, ``forward`` runs the wrapped layers."""

    def __init__(self, layers, hcg, strategy=None):
        super().__init__()
        self._layers = layers
        self._hcg = hcg
        self._strategy = strategy
        self._grad_sync = None
        self._prepare_for_model()

    def _prepare_for_model(self):
        pass

    def _install_grad_sync(self):
        """dp / sep gradient all-reduce overlapped with backward (hybrid_parallel_util.install_grad_sync)."""
        from ..utils.hybrid_parallel_util import install_grad_sync
        mb = getattr(self._strategy, 'fuse_grad_size_in_MB', 64) if self._strategy is not None else 64
        self._grad_sync = install_grad_sync(self._layers, self._hcg, mb or 64)

    def forward(self, *a, **k):
        return self._layers(*a, **k)

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layers.set_state_dict(*a, **k)


class TensorParallel(MetaParallelBase):
    """Model built from mpu layers: replicated (non-distributed) parameters agree over mp; the
    whole model is broadcast over sep / sharding / dp (reference tensor_parallel.py:29-47)."""

    def _prepare_for_model(self):
        import torch
        import torch.distributed as dist
        from ..utils.hybrid_parallel_util import (broadcast_dp_parameters, broadcast_sep_parameters,
                                                  broadcast_sharding_parameters)
        hcg = self._hcg
        g = hcg.get_model_parallel_group()
        if g is not None and g.nranks > 1:
            with torch.no_grad():
                for p in self._layers.parameters():
                    if not getattr(p, 'is_distributed', False):
                        dist.broadcast(p._t, hcg.get_model_parallel_group_src_rank(), group=g.pg)
        if hcg.get_sep_parallel_world_size() > 1:
            broadcast_sep_parameters(self._layers, hcg)
        if hcg.get_sharding_parallel_world_size() > 1:
            broadcast_sharding_parameters(self._layers, hcg)
        broadcast_dp_parameters(self._layers, hcg)
        if hcg.get_sharding_parallel_world_size() == 1:
            # a sharding optimizer reduces over dp on its shards itself
            self._install_grad_sync()


class SegmentParallel(MetaParallelBase):
    """Sequence split over the ``sep`` axis (reference segment_parallel.py:26-40): every sep rank
    runs the same weights on its own segment of each sequence (the model exchanges activations
    with its sep peers, e.g. by all-to-all / all-gather), so the weights are broadcast over sep,
    sharding and dp, and the gradients are SUMMED over sep and averaged over dp — during backward,
    by a hook-driven bucketed all-reduce on the dp x sep group."""

    def _prepare_for_model(self):
        from ..utils.hybrid_parallel_util import (broadcast_dp_parameters, broadcast_sep_parameters,
                                                  broadcast_sharding_parameters)
        hcg = self._hcg
        broadcast_sep_parameters(self._layers, hcg)
        if hcg.get_sharding_parallel_world_size() > 1:
            broadcast_sharding_parameters(self._layers, hcg)
        if hcg.get_data_parallel_world_size() > 1:
            broadcast_dp_parameters(self._layers, hcg)
        if hcg.get_sharding_parallel_world_size() == 1:
            self._install_grad_sync()


class ShardingParallel(MetaParallelBase):
    """Sharding axis only (reference sharding_parallel.py): parameters broadcast over sharding
    and dp; gradients are reduce-scattered by the sharding optimizer."""

    def _prepare_for_model(self):
        from ..utils.hybrid_parallel_util import broadcast_dp_parameters, broadcast_sharding_parameters
        broadcast_sharding_parameters(self._layers, self._hcg)
        broadcast_dp_parameters(self._layers, self._hcg)
