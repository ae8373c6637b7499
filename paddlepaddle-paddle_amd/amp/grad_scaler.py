"""GradScaler (reference: python/paddle/amp/grad_scaler.py).

Dynamic loss scaling: ``scale(loss)`` multiplies by the current scale; ``minimize``/``step``
unscales the gradients with one fused multi-tensor pass, checks for inf/nan (one
device-side reduction, one host sync), skips the update on overflow and adapts the scale.
"""
import enum

import torch

from ..core.tensor import Tensor, _wrap, _unwrap


class OptimizerState(enum.Enum):
    INIT = 0
    UNSCALED = 1
    STEPPED = 2


class AmpScaler:
    def __init__(self, enable=True, init_loss_scaling=65536.0, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=2000, decr_every_n_nan_or_inf=1, use_dynamic_loss_scaling=True):
        self._enable = enable
        self._scale = float(init_loss_scaling)
        self._incr_ratio, self._decr_ratio = incr_ratio, decr_ratio
        self._incr_every, self._decr_every = incr_every_n_steps, decr_every_n_nan_or_inf
        self._dynamic = use_dynamic_loss_scaling
        self._good, self._bad = 0, 0
        self._found_inf = False
        self._opt_state = {}

    def is_enable(self):
        return self._enable

    def is_use_dynamic_loss_scaling(self):
        return self._dynamic

    def get_init_loss_scaling(self):
        return self._scale

    def set_init_loss_scaling(self, v):
        self._scale = float(v)

    def scale(self, var):
        if not self._enable:
            return var
        return _wrap(_unwrap(var) * self._scale)

    def _unscale(self, optimizer):
        if not self._enable:
            return
        st = self._opt_state.get(id(optimizer), OptimizerState.INIT)
        if st == OptimizerState.UNSCALED:
            return
        engine = getattr(optimizer, 'engine', None)
        if engine is not None and hasattr(engine, 'arenas'):  # sharded optimizer: its gradients live in the arenas
            grads = [a['grad'] for a in engine.arenas.values()]
        else:
            grads = [p._t.grad for p in optimizer._parameter_list if p._t.grad is not None]
        if not grads:
            self._found_inf = self._sync_found_inf(False)
            return
        inv = 1.0 / self._scale
        found = torch.zeros((), dtype=torch.float32, device=grads[0].device)
        by_dev = {}
        for g in grads:
            by_dev.setdefault((g.device, g.dtype), []).append(g)
        for (dev, dt), gs in by_dev.items():
            torch._foreach_mul_(gs, inv)
            fi = torch.zeros((), dtype=torch.float32, device=dev)
            torch._amp_foreach_non_finite_check_and_unscale_(gs, fi, torch.ones((), device=dev)) \
                if dev.type == 'cuda' else fi.add_(sum(float(~torch.isfinite(g).all()) for g in gs))
            found = found + fi.to(found.device)
        self._found_inf = self._sync_found_inf(found)
        self._opt_state[id(optimizer)] = OptimizerState.UNSCALED

    def _sync_found_inf(self, found):
        """Hook for distributed scalers (fleet.distributed_scaler): every rank must agree."""
        if isinstance(found, bool):
            return found
        return bool(found.item() > 0)

    def unscale_(self, optimizer):
        self._unscale(optimizer)

    def minimize(self, optimizer, *args, **kwargs):
        if not self._enable:
            return optimizer.minimize(*args, **kwargs)
        self._unscale(optimizer)
        if not self._found_inf:
            optimizer.step()
        self._update()
        self._opt_state.clear()
        return None, None

    def step(self, optimizer):
        if not self._enable:
            return optimizer.step()
        self._unscale(optimizer)
        if not self._found_inf:
            optimizer.step()
        self._opt_state[id(optimizer)] = OptimizerState.STEPPED

    def update(self):
        if not self._enable:
            return
        self._update()
        self._opt_state.clear()

    def _update(self):
        if not self._dynamic:
            return
        if self._found_inf:
            self._bad += 1
            self._good = 0
            if self._bad >= self._decr_every:
                self._scale = max(self._scale * self._decr_ratio, 1.0)
                self._bad = 0
        else:
            self._good += 1
            self._bad = 0
            if self._good >= self._incr_every:
                self._scale *= self._incr_ratio
                self._good = 0

    def state_dict(self):
        return {'scale': _wrap(torch.tensor([self._scale])), 'incr_ratio': self._incr_ratio,
                'decr_ratio': self._decr_ratio, 'incr_every_n_steps': self._incr_every,
                'decr_every_n_nan_or_inf': self._decr_every, 'incr_count': self._good, 'decr_count': self._bad,
                'use_dynamic_loss_scaling': self._dynamic}

    def load_state_dict(self, state_dict):
        s = state_dict['scale']
        self._scale = float(s.numpy().reshape(-1)[0]) if hasattr(s, 'numpy') else float(s)
        self._good = state_dict.get('incr_count', 0)
        self._bad = state_dict.get('decr_count', 0)

    set_state_dict = load_state_dict


class GradScaler(AmpScaler):
    def __init__(self, enable=True, init_loss_scaling=2.0 ** 16, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=2000, decr_every_n_nan_or_inf=1, use_dynamic_loss_scaling=True):
        super().__init__(enable, init_loss_scaling, incr_ratio, decr_ratio, incr_every_n_steps,
                         decr_every_n_nan_or_inf, use_dynamic_loss_scaling)
