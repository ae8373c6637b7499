"""Optimizer base (reference: python/paddle/optimizer/optimizer.py:104).

* parameter groups (list of Parameters or list of dicts with per-group overrides)
* grad clipping (``grad_clip``) and L1/L2 regularisation (``weight_decay``) semantics of paddle
* accumulators named like the reference (``{param.name}_moment1_0`` …) so ``state_dict``
  round-trips through ``.pdopt`` files
* multi_precision: fp32 master weights for bf16/fp16 parameters
* GPU fast path (Adam/AdamW): parameters are re-homed into flat buffers (parallel.flat_buffer)
  and the whole update is one fused HIP kernel per dtype group.
"""
import collections

import numpy as np
import torch

from ..core.tensor import Tensor, Parameter, _wrap, _unwrap
from ..regularizer import L1Decay, L2Decay, WeightDecayRegularizer
from .lr import LRScheduler


class Optimizer:
    _acc_names = ()

    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, name=None):
        if parameters is not None and isinstance(parameters, (Tensor,)):
            raise TypeError("parameters should be a list of Parameters or param-group dicts")
        self._learning_rate = learning_rate
        self._grad_clip = grad_clip
        self._name = name
        self.regularization = None
        if isinstance(weight_decay, float) or isinstance(weight_decay, int):
            self.regularization = L2Decay(float(weight_decay)) if weight_decay else None
            self._weight_decay = float(weight_decay)
        else:
            self.regularization = weight_decay
            self._weight_decay = weight_decay
        self._param_groups = []
        if parameters is not None:
            parameters = list(parameters)
            if parameters and isinstance(parameters[0], dict):
                for g in parameters:
                    self._add_param_group(dict(g))
            else:
                self._add_param_group({'params': parameters})
        self._parameter_list = [p for g in self._param_groups for p in g['params']]
        self._accumulators = collections.defaultdict(dict)  # acc_name -> {param_name: torch tensor}
        self._master_weights = {}
        self._global_step = 0
        self.helper = None

    # ------------------------------------------------------------------ groups
    def _add_param_group(self, group):
        params = group['params']
        if isinstance(params, Tensor):
            params = [params]
        group['params'] = list(params)
        group.setdefault('learning_rate', 1.0)
        self._param_groups.append(group)

    def add_param_group(self, param_group):
        self._add_param_group(dict(param_group))
        self._parameter_list = [p for g in self._param_groups for p in g['params']]

    # ------------------------------------------------------------------ lr
    def get_lr(self):
        lr = self._learning_rate
        return float(lr()) if isinstance(lr, LRScheduler) else float(lr)

    def set_lr(self, value):
        if isinstance(self._learning_rate, LRScheduler):
            raise RuntimeError("optimizer's learning rate can't be LRScheduler when invoke this API")
        self._learning_rate = float(value)

    def set_lr_scheduler(self, scheduler):
        self._learning_rate = scheduler

    # ------------------------------------------------------------------ accumulators
    def _acc(self, name, p, fill=0.0, dtype=torch.float32, shape=None):
        d = self._accumulators[name]
        t = d.get(p.name)
        if t is None:
            t = torch.full(shape if shape is not None else p._t.shape, fill, dtype=dtype, device=p._t.device)
            d[p.name] = t
        return t

    def _master(self, p):
        if p._t.dtype in (torch.float16, torch.bfloat16) and self._multi_precision:
            m = self._master_weights.get(p.name)
            if m is None:
                m = p._t.detach().float().clone()
                self._master_weights[p.name] = m
            return m
        return None

    _multi_precision = False

    # ------------------------------------------------------------------ API
    def clear_grad(self, set_to_zero=True):
        for p in self._parameter_list:
            if set_to_zero:
                if p._t.grad is not None:
                    p._t.grad.zero_()
            else:
                if '_flat' in p.__dict__:
                    if p._t.grad is not None:
                        p._t.grad.zero_()
                else:
                    p._t.grad = None

    clear_gradients = clear_grad

    def _params_grads(self, group):
        out = []
        for p in group['params']:
            if not p.trainable or p._t.grad is None:
                continue
            out.append((p, _wrap(p._t.grad)))
        return out

    def _apply_regularization(self, p, g, group):
        reg = group.get('weight_decay', self.regularization)
        if isinstance(reg, (int, float)):
            reg = L2Decay(float(reg)) if reg else None
        if getattr(p, 'regularizer', None) is not None:
            reg = p.regularizer
        if reg is None:
            return g
        if isinstance(reg, L2Decay):
            return g + reg._coeff * p._t.detach().to(g.dtype)
        if isinstance(reg, L1Decay):
            return g + reg._coeff * torch.sign(p._t.detach()).to(g.dtype)
        return g

    @torch.no_grad()
    def step(self):
        lr = self.get_lr()
        for group in self._param_groups:
            pg = self._params_grads(group)
            if not pg:
                continue
            clip = group.get('grad_clip', self._grad_clip)
            if clip is not None:
                pg = clip(pg)
            glr = lr * group.get('learning_rate', 1.0)
            self._update_group(group, pg, glr)
        self._global_step += 1

    def _update_group(self, group, params_grads, lr):
        for p, g in params_grads:
            plr = lr * p.__dict__.get('optimize_attr', {}).get('learning_rate', 1.0)
            self._update_param(p, g._t, plr, group)

    def _update_param(self, p, g, lr, group):
        raise NotImplementedError

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ..framework import in_dynamic_mode
        if not in_dynamic_mode():
            from ..static.program import _static_minimize
            return _static_minimize(self, loss, parameters, no_grad_set)
        if parameters is not None and not self._parameter_list:
            self._add_param_group({'params': list(parameters)})
            self._parameter_list = list(parameters)
        loss.backward()
        self.step()
        return None, None

    # ------------------------------------------------------------------ state
    def state_dict(self):
        sd = collections.OrderedDict()
        for acc, d in self._accumulators.items():
            for pname, t in d.items():
                sd[f"{pname}_{acc}_0"] = _wrap(t)
        for pname, t in self._master_weights.items():
            sd.setdefault('master_weights', collections.OrderedDict())[pname] = _wrap(t)
        if isinstance(self._learning_rate, LRScheduler):
            sd['LR_Scheduler'] = self._learning_rate.state_dict()
        sd['@global_step@'] = self._global_step
        return sd

    def set_state_dict(self, state_dict):
        if 'LR_Scheduler' in state_dict and isinstance(self._learning_rate, LRScheduler):
            self._learning_rate.set_state_dict(state_dict['LR_Scheduler'])
        self._global_step = int(state_dict.get('@global_step@', self._global_step))
        names = {p.name: p for p in self._parameter_list}
        for k, v in state_dict.items():
            if k in ('LR_Scheduler', '@global_step@'):
                continue
            if k == 'master_weights':
                for pn, t in v.items():
                    src = _to_torch(t)
                    self._master_weights[pn] = src.to(names[pn]._t.device).float() if pn in names else src.float()
                continue
            for acc in self._acc_names:
                suffix = f"_{acc}_0"
                if k.endswith(suffix):
                    pname = k[:-len(suffix)]
                    dev = names[pname]._t.device if pname in names else 'cpu'
                    self._accumulators[acc][pname] = _to_torch(v).to(dev)
        self._on_state_loaded()

    def _on_state_loaded(self):
        pass

    set_dict = set_state_dict

    def __repr__(self):
        return f"{self.__class__.__name__}(lr={self.get_lr()})"


def _to_torch(v):
    if isinstance(v, Tensor):
        return v._t.detach().clone()
    if isinstance(v, tuple) and len(v) == 2:
        v = v[1]
    a = np.asarray(v)
    if a.dtype == np.uint16:
        return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
    return torch.from_numpy(a.copy())
