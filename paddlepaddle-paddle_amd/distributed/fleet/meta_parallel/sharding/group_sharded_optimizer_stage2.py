"""GroupShardedOptimizerStage2 (reference: meta_parallel/sharding/group_sharded_optimizer_stage2.py:53).

In the reference the optimizer is constructed first and the model wrapper (GroupShardedStage2)
second; the sharding engine needs the model, so this object records the optimizer and group, and
GroupShardedStage2 binds the engine (parallel/sharding.ShardedOptimizer) into it.  Until then the
inner optimizer is used as is."""


class GroupShardedOptimizerStage2:
    def __init__(self, params, optim, group=None, offload=False, device="gpu", pretrain_sync_models=True,
                 dp_group=None, **kw):
        self._optim = optim
        self._params = list(params) if params is not None else list(optim._parameter_list)
        self._group = group
        self._dp_group = dp_group
        self._sharded = None  # parallel.sharding.ShardedOptimizer, set by GroupShardedStage2
        self.offload = bool(offload)  # read by GroupShardedStage2 when it builds the engine

    def _bind(self, sharded):
        self._sharded = sharded

    @property
    def _target(self):
        return self._sharded if self._sharded is not None else self._optim

    def step(self):
        return self._target.step()

    def clear_grad(self, set_to_zero=True):
        return self._target.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def minimize(self, loss, *a, **k):
        loss.backward()
        self.step()

    def state_dict(self):
        return self._target.state_dict()

    def set_state_dict(self, sd):
        return self._target.set_state_dict(sd)

    def get_lr(self):
        return self._optim.get_lr()

    def set_lr(self, v):
        return self._optim.set_lr(v)

    @property
    def _parameter_list(self):
        return self._params

    def __getattr__(self, name):
        return getattr(self.__dict__['_optim'], name)
