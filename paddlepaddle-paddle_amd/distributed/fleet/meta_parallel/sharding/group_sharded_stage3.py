"""GroupShardedStage3 (reference: meta_parallel/sharding/group_sharded_stage3.py:85): parameters,
gradients and optimizer state sharded ('p_g_os' of parallel/sharding.ShardingEngine: one flat unit
per layer block, all-gathered before the block runs, released after; gradients reduce-scattered
as backward produces them).  The user's optimizer object keeps working: its step / clear_grad /
state_dict are rebound to the sharded update of the engine's arena."""
from .....nn.layer.layers import Layer
from .....parallel.sharding import ShardingEngine, ShardedOptimizer, gathered_state_dict


class GroupShardedStage3(Layer):
    def __init__(self, layer, optimizer, group=None, sync_buffers=False, device="gpu", segment_size=2 ** 20,
                 pretrain_sync_models=True, offload=False, sync_comm=False, dp_group=None, exclude_layer=None):
        super().__init__()
        self._layer = layer
        # offload: the shard's fp32 master + Adam moments in pinned host memory, updated by the host
        # runtime (parallel/sharding.py ShardingEngine offload)
        engine = ShardingEngine(layer, 'p_g_os', group=group, segment_size=segment_size, offload=offload)
        self.__dict__['_engine'] = engine
        inner = optimizer._optim if hasattr(optimizer, '_bind') else optimizer
        sharded = ShardedOptimizer(inner, engine)
        if hasattr(optimizer, '_bind'):
            optimizer._bind(sharded)
        else:  # rebind the plain optimizer's entry points onto the sharded update
            optimizer.step = sharded.step
            optimizer.clear_grad = sharded.clear_grad
            optimizer.clear_gradients = sharded.clear_grad
            optimizer.state_dict = sharded.state_dict
            optimizer.set_state_dict = sharded.set_state_dict
        self._optim = optimizer
        self._sharded = sharded

    def forward(self, *a, **k):
        return self._layer(*a, **k)

    def get_all_parameters(self, convert2cpu=False):
        eng = self.__dict__['_engine']
        eng.wait_param_gathers()
        for u in eng.units:
            u.wait_gather()
        ps = self._layer.parameters()
        if convert2cpu:
            for p in ps:
                p._t.data = p._t.data.cpu()
        return ps

    def state_dict(self, *a, **k):
        return gathered_state_dict(self._layer, self.__dict__['_engine'])

    def set_state_dict(self, sd, use_structured_name=True):
        return self._layer.set_state_dict(sd, use_structured_name)
