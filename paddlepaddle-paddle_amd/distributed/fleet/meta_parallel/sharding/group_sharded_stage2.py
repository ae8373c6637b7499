"""GroupShardedStage2 (reference: meta_parallel/sharding/group_sharded_stage2.py:46): gradients
reduce-scattered per unit as backward produces them, optimizer state sharded (stage 2 'os_g' of
parallel/sharding.ShardingEngine)."""
from .....nn.layer.layers import Layer
from .....parallel.sharding import ShardingEngine, ShardedOptimizer, gathered_state_dict


class GroupShardedStage2(Layer):
    def __init__(self, layer, sharding_optimizer, group=None, sync_buffers=False, buffer_max_size=2 ** 23,
                 auto_refresh_trainable=True, device="gpu", dp_group=None):
        super().__init__()
        self._layer = layer
        opts = sharding_optimizer if isinstance(sharding_optimizer, list) else [sharding_optimizer]
        self._sharding_optimizers = opts
        engine = ShardingEngine(layer, 'os_g', group=group,
                                bucket_mb=max(1, int(buffer_max_size * 2 // 2 ** 20)) if buffer_max_size else 256,
                                offload=any(getattr(o, 'offload', False) for o in opts))
        self.__dict__['_engine'] = engine
        for o in opts:
            inner = o._optim if hasattr(o, '_bind') else o
            sharded = ShardedOptimizer(inner, engine)
            if hasattr(o, '_bind'):
                o._bind(sharded)

    def forward(self, *a, **k):
        return self._layer(*a, **k)

    def state_dict(self, *a, **k):
        return gathered_state_dict(self._layer, self.__dict__['_engine'])

    def set_state_dict(self, sd, use_structured_name=True):
        return self._layer.set_state_dict(sd, use_structured_name)
