"""Optimizer algorithms (reference: python/paddle/optimizer/{sgd,momentum,adam,adamw,adamax,adagrad,
adadelta,rmsprop,lamb,nadam,radam,asgd,rprop,lbfgs}.py and the phi update kernels).

Update math follows the phi kernels (e.g. paddle's Adam scales epsilon by sqrt(1 - beta2^t)).
"""
import math

import torch

from ..core.tensor import Tensor, _wrap, _unwrap
from .optimizer import Optimizer
from .. import ops


def _write_back(p, new_fp32, master):
    if master is not None:
        master.copy_(new_fp32)
        p._t.data.copy_(new_fp32.to(p._t.dtype))
    else:
        p._t.data.copy_(new_fp32.to(p._t.dtype))


class SGD(Optimizer):
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, multi_precision=False,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._multi_precision = multi_precision

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group)
        m = self._master(p)
        if m is not None:
            m.add_(g.float(), alpha=-lr)
            p._t.data.copy_(m.to(p._t.dtype))
        else:
            p._t.data.add_(g.to(p._t.dtype), alpha=-lr)


class Momentum(Optimizer):
    _acc_names = ('velocity',)

    def __init__(self, learning_rate=0.001, momentum=0.9, parameters=None, use_nesterov=False, weight_decay=None,
                 grad_clip=None, multi_precision=False, rescale_grad=1.0, use_multi_tensor=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._momentum, self._use_nesterov, self._rescale = momentum, use_nesterov, rescale_grad
        self._multi_precision = multi_precision

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float() * self._rescale
        v = self._acc('velocity', p)
        v.mul_(self._momentum).add_(g)
        m = self._master(p)
        base = m if m is not None else p._t.data.float()
        upd = (g + self._momentum * v) if self._use_nesterov else v
        _write_back(p, base - lr * upd, m)

    # ---- fused flat path (GPU): one csrc momentum kernel per (dtype, L2 coeff) bucket instead of
    # ~8 elementwise launches per parameter (ResNet50: 161 parameters)
    _flat = None

    def _l2(self, p, group):
        from ..regularizer import L2Decay
        reg = group.get('weight_decay', self.regularization)
        if isinstance(reg, (int, float)):
            return float(reg)
        if reg is None:
            return 0.0
        return float(reg._coeff) if isinstance(reg, L2Decay) else None

    def _fusable(self):
        if not self._parameter_list or not ops.use_hip(self._parameter_list[0]._t):
            return False
        for group in self._param_groups:
            if self._l2(None, group) is None:
                return False
        for p in self._parameter_list:
            if p._t.device.type != 'cuda' or getattr(p, 'regularizer', None) is not None:
                return False
            if p.__dict__.get('optimize_attr', {}).get('learning_rate', 1.0) != 1.0:
                return False
        return True

    def _build_flat(self):
        from ..parallel.flat_buffer import FlatBuffer
        self._flat = []
        for gi, group in enumerate(self._param_groups):
            buckets = {}
            for p in group['params']:
                if p.trainable:
                    buckets.setdefault(p._t.dtype, []).append(p)
            for dt, ps in buckets.items():
                fb = ps[0].__dict__.get('_flat', (None,))[0]
                if fb is None or set(map(id, fb.params)) != set(map(id, ps)):
                    fb = FlatBuffer(ps)
                master = fb.data.float().clone() if dt != torch.float32 else fb.data
                vel = torch.zeros(fb.numel, dtype=torch.float32, device=fb.device)
                self._flat.append({'fb': fb, 'master': master, 'v': vel, 'l2': self._l2(None, group), 'group': gi})
                for p, o in zip(fb.params, fb.offsets):
                    n = p._t.numel()
                    self._accumulators['velocity'][p.name] = vel[o:o + n].view(p._t.shape)
                    if dt != torch.float32:
                        self._master_weights[p.name] = master[o:o + n].view(p._t.shape)

    def step(self):
        if self._flat is None and self._fusable():
            self._build_flat()
        if self._flat is None:
            return super().step()
        with torch.no_grad():
            for ent in self._flat:
                if not ent['fb'].data_intact():
                    self._flat = None
                    return super().step()
                ent['fb'].sync_grads()
            for group in self._param_groups:
                clip = group.get('grad_clip', self._grad_clip)
                if clip is not None:
                    clip(self._params_grads(group))
            lr = self.get_lr()
            dev_lr = _graph_lr(self, self._flat, self._advance_host_step)
            for ent in self._flat:
                fb = ent['fb']
                glr = lr * self._param_groups[ent['group']].get('learning_rate', 1.0)
                ops.optim.momentum_flat(ent['master'], fb.grad, ent['v'], fb.data if fb.dtype != torch.float32 else None,
                                        glr, self._momentum, ent['l2'], self._rescale, self._use_nesterov,
                                        lr_tensor=ent['lr_dev'] if dev_lr else None)
        self._global_step += 1

    def _advance_host_step(self):
        self._global_step += 1

    def clear_grad(self, set_to_zero=True):
        if self._flat is None:
            return super().clear_grad(set_to_zero)
        for fb in {id(e['fb']): e['fb'] for e in self._flat}.values():
            fb.grad.zero_()
        for p in self._parameter_list:
            if '_flat' not in p.__dict__ and p._t.grad is not None:
                p._t.grad.zero_()

    clear_gradients = clear_grad


class Adam(Optimizer):
    _acc_names = ('moment1', 'moment2', 'beta1_pow_acc', 'beta2_pow_acc')
    _decoupled = False

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None, weight_decay=None,
                 grad_clip=None, lazy_mode=False, multi_precision=False, use_multi_tensor=True, amsgrad=False,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._beta1 = float(_unwrap(beta1).item()) if isinstance(beta1, Tensor) else beta1
        self._beta2 = float(_unwrap(beta2).item()) if isinstance(beta2, Tensor) else beta2
        self._epsilon = float(_unwrap(epsilon).item()) if isinstance(epsilon, Tensor) else epsilon
        self._multi_precision = multi_precision
        self._use_fused = use_multi_tensor
        self._amsgrad = amsgrad
        self._flat = None  # list of fused groups

    # ---- per-parameter reference path (CPU, or anything the fused path does not cover)
    def _decay_coeff(self, p, group):
        return 0.0

    def _update_param(self, p, g, lr, group):
        b1, b2, eps = self._beta1, self._beta2, self._epsilon
        if not self._decoupled:
            g = self._apply_regularization(p, g, group)
        g = g.float()
        m1 = self._acc('moment1', p)
        m2 = self._acc('moment2', p)
        b1p = self._acc('beta1_pow_acc', p, fill=b1, shape=[1])
        b2p = self._acc('beta2_pow_acc', p, fill=b2, shape=[1])
        master = self._master(p)
        pv = master if master is not None else p._t.data.float()
        coeff = self._decay_coeff(p, group)
        if coeff:
            pv = pv * (1.0 - lr * coeff)
        m1.mul_(b1).add_(g, alpha=1 - b1)
        m2.mul_(b2).addcmul_(g, g, value=1 - b2)
        if self._amsgrad:
            mx = self._acc('moment2_max', p)
            torch.maximum(mx, m2, out=mx)
            denom_src = mx
        else:
            denom_src = m2
        bc2 = torch.sqrt(1 - b2p)
        lr_t = lr * bc2 / (1 - b1p)
        pv = pv - lr_t * m1 / (denom_src.sqrt() + eps * bc2)
        _write_back(p, pv, master)
        b1p.mul_(b1)
        b2p.mul_(b2)

    # ---- fused flat path (GPU)
    def _fusable(self):
        if not self._use_fused or self._amsgrad:
            return False
        for p in self._parameter_list:
            if p._t.device.type != 'cuda' or getattr(p, 'regularizer', None) is not None:
                return False
            if p.__dict__.get('optimize_attr', {}).get('learning_rate', 1.0) != 1.0:
                return False
        if not self._decoupled and self.regularization is not None:
            return False
        return bool(self._parameter_list) and ops.use_hip(self._parameter_list[0]._t)

    def _build_flat(self):
        from ..parallel.flat_buffer import FlatBuffer
        self._flat = []
        for gi, group in enumerate(self._param_groups):
            buckets = {}
            for p in group['params']:
                if not p.trainable:
                    continue
                key = (p._t.dtype, self._decay_coeff(p, group))
                buckets.setdefault(key, []).append(p)
            for (dt, coeff), ps in buckets.items():
                fb = ps[0].__dict__.get('_flat', (None,))[0]
                if fb is None or set(map(id, fb.params)) != set(map(id, ps)):
                    fb = FlatBuffer(ps)
                master = fb.data.float().clone() if dt != torch.float32 else fb.data
                m1 = torch.zeros_like(master) if dt != torch.float32 else torch.zeros(fb.numel, device=fb.device)
                m2 = torch.zeros_like(m1)
                ent = {'fb': fb, 'master': master, 'm1': m1, 'm2': m2, 'coeff': coeff, 'group': gi,
                       'b1p': self._beta1, 'b2p': self._beta2}
                self._flat.append(ent)
                for p, o in zip(fb.params, fb.offsets):
                    n = p._t.numel()
                    self._accumulators['moment1'][p.name] = m1[o:o + n].view(p._t.shape)
                    self._accumulators['moment2'][p.name] = m2[o:o + n].view(p._t.shape)
                    if dt != torch.float32:
                        self._master_weights[p.name] = master[o:o + n].view(p._t.shape)

    def step(self):
        if self._flat is None and self._fusable():
            self._build_flat()
        if self._flat is None:
            return super().step()
        with torch.no_grad():
            lr = self.get_lr()
            for ent in self._flat:
                fb = ent['fb']
                if not fb.data_intact():
                    # parameters were re-homed (e.g. Layer.to()); fall back permanently
                    self._flat = None
                    return super().step()
                fb.sync_grads()
            scale = self._clip_flat()
            capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
            dev_lr = _graph_lr(self, self._flat, self._advance_host_step)
            for ent in self._flat:
                fb = ent['fb']
                glr = lr * self._param_groups[ent['group']].get('learning_rate', 1.0)
                lowp = fb.data if fb.dtype != torch.float32 else None
                pows = _device_pows(ent, self._beta1, self._beta2, fb.device, capturing)
                ops.optim.adamw_flat(ent['master'], fb.grad, ent['m1'], ent['m2'], lowp, glr, self._beta1,
                                     self._beta2, self._epsilon, ent['coeff'], ent['b1p'], ent['b2p'],
                                     lr_tensor=ent['lr_dev'] if dev_lr else None,
                                     grad_scale=scale, pows=pows if capturing else None)
                ent['b1p'] *= self._beta1
                ent['b2p'] *= self._beta2
                if pows is not None:
                    pows.mul_(ent['betas'])
                    ent['graph_stepped'] = ent.get('graph_stepped', False) or capturing
        self._global_step += 1

    def _advance_host_step(self):
        # a replay of a captured step: the device powers advanced in the graph, the host copies here
        for ent in self._flat or ():
            ent['b1p'] *= self._beta1
            ent['b2p'] *= self._beta2
        self._global_step += 1

    def _clip_flat(self):
        """Global-norm clip over the flat gradient buffers: one sum-of-squares kernel per buffer;
        the resulting scale is returned and applied inside the AdamW kernel's gradient read
        (no separate scaling pass).  Non-global clips are applied eagerly and return None."""
        from ..nn.clip import ClipGradByGlobalNorm
        clips = {id(g.get('grad_clip', self._grad_clip)): g.get('grad_clip', self._grad_clip)
                 for g in self._param_groups}
        clips = [c for c in clips.values() if c is not None]
        if not clips:
            return
        if len(clips) > 1 or not isinstance(clips[0], ClipGradByGlobalNorm):
            for group in self._param_groups:
                clip = group.get('grad_clip', self._grad_clip)
                if clip is not None:
                    clip(self._params_grads(group))
            return
        clip = clips[0]
        bufs = {id(e['fb']): e['fb'] for e in self._flat}.values()
        sq = None
        for fb in bufs:
            s = ops.optim.sumsq(fb.grad)
            sq = s if sq is None else sq + s
        if clip._extra_sq_norm_fn is not None:
            sq = clip._extra_sq_norm_fn(sq)
        return torch.clamp(clip.clip_norm / torch.clamp(sq.sqrt(), min=clip.clip_norm), max=1.0)

    def clear_grad(self, set_to_zero=True):
        if self._flat is None:
            return super().clear_grad(set_to_zero)
        for fb in {id(e['fb']): e['fb'] for e in self._flat}.values():
            fb.grad.zero_()
        for p in self._parameter_list:  # parameters outside the flat buffers
            if '_flat' not in p.__dict__ and p._t.grad is not None:
                p._t.grad.zero_()

    clear_gradients = clear_grad

    def state_dict(self):
        sd = super().state_dict()
        if self._flat is not None:
            for ent in self._flat:
                # the fp64 host powers: advanced by every eager step and, through the replay hook
                # (_advance_host_step), by every graph replay too — one checkpoint precision
                # whether or not the run replayed (the fp32 device copy is for the kernel only)
                b1p, b2p = ent['b1p'], ent['b2p']
                for p in ent['fb'].params:
                    sd[f"{p.name}_beta1_pow_acc_0"] = _wrap(torch.tensor([b1p]))
                    sd[f"{p.name}_beta2_pow_acc_0"] = _wrap(torch.tensor([b2p]))
        return sd

    def _on_state_loaded(self):
        if self._flat is None:
            return
        with torch.no_grad():
            for ent in self._flat:
                fb = ent['fb']
                for p, o in zip(fb.params, fb.offsets):
                    n = p._t.numel()
                    for acc, buf in (('moment1', ent['m1']), ('moment2', ent['m2'])):
                        t = self._accumulators[acc].get(p.name)
                        if t is not None and t.data_ptr() != buf[o:o + 1].data_ptr():
                            buf[o:o + n].copy_(t.reshape(-1))
                            self._accumulators[acc][p.name] = buf[o:o + n].view(p._t.shape)
                    mw = self._master_weights.get(p.name)
                    if mw is not None and fb.dtype != torch.float32 and mw.data_ptr() != ent['master'][o:o + 1].data_ptr():
                        ent['master'][o:o + n].copy_(mw.reshape(-1))
                        self._master_weights[p.name] = ent['master'][o:o + n].view(p._t.shape)
                    b1 = self._accumulators['beta1_pow_acc'].get(p.name)
                    if b1 is not None:
                        ent['b1p'] = float(b1.reshape(-1)[0])
                    b2 = self._accumulators['beta2_pow_acc'].get(p.name)
                    if b2 is not None:
                        ent['b2p'] = float(b2.reshape(-1)[0])
                if ent.get('pows') is not None:
                    ent['pows'].copy_(torch.tensor([ent['b1p'], ent['b2p']]))


def _graph_lr(opt, ents, post):
    """Learning rate as a device scalar for a step being captured by a TrainStepGraph
    (device/cuda/graphs.py on_replay): each flat-buffer entry holds an fp32 [1] ``lr_dev`` that the
    graph's pre-replay hook refills from ``opt.get_lr()`` (times the group multiplier), so a host
    LR scheduler keeps working across replays; ``post`` advances the optimizer's host counters
    after each replay.  False (use the host value) when nothing is being captured that way.

    ``lr_dev`` is allocated on an eager step, never inside the capture: a block taken from the
    graph's private pool may be one a temporary earlier in the same step used, which the replay
    would overwrite after the pre-replay fill."""
    if not torch.cuda.is_available():
        return False
    if not torch.cuda.is_current_stream_capturing():
        for ent in ents:
            if ent.get('lr_dev') is None and ent['fb'].device.type == 'cuda':
                ent['lr_dev'] = torch.zeros(1, dtype=torch.float32, device=ent['fb'].device)
        return False
    if any(ent.get('lr_dev') is None for ent in ents):
        return False  # captured without an eager step first: host value (frozen)
    from ..device.cuda.graphs import on_replay

    def pre():
        lr = opt.get_lr()
        for ent in ents:
            ent['lr_dev'].fill_(lr * opt._param_groups[ent['group']].get('learning_rate', 1.0))
    return on_replay(pre=pre, post=post)


def _device_pows(ent, b1, b2, device, capturing):
    """Device copy [beta1^t, beta2^t] of a flat entry's bias-correction powers, advanced on the
    device after every update (eager steps keep reading the host values): a training step captured
    into a hipGraph (device/cuda/graphs.py TrainStepGraph) reads and advances it, so replays see
    the powers of their own step instead of the ones frozen at capture.  Created on the first
    eager step (never inside a capture)."""
    pows = ent.get('pows')
    if pows is None and not capturing and str(device).startswith('cuda'):
        pows = ent['pows'] = torch.tensor([ent['b1p'], ent['b2p']], dtype=torch.float32, device=device)
        ent['betas'] = torch.tensor([b1, b2], dtype=torch.float32, device=device)
    return pows


class AdamW(Adam):
    _decoupled = True

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None, weight_decay=0.01,
                 lr_ratio=None, apply_decay_param_fun=None, grad_clip=None, lazy_mode=False, multi_precision=False,
                 amsgrad=False, name=None):
        super().__init__(learning_rate, beta1, beta2, epsilon, parameters, None, grad_clip, lazy_mode,
                         multi_precision, True, amsgrad, name)
        self._coeff = float(_unwrap(weight_decay).item()) if isinstance(weight_decay, Tensor) else float(weight_decay)
        self._apply_decay_param_fun = apply_decay_param_fun
        self._lr_ratio = lr_ratio
        if lr_ratio is not None:
            self._use_fused = False

    def _decay_coeff(self, p, group):
        if self._apply_decay_param_fun is not None and not self._apply_decay_param_fun(p.name):
            return 0.0
        return float(group.get('weight_decay', self._coeff) or 0.0)

    def _update_param(self, p, g, lr, group):
        if self._lr_ratio is not None:
            lr = lr * self._lr_ratio(p)
        super()._update_param(p, g, lr, group)


class Adamax(Optimizer):
    _acc_names = ('moment', 'inf_norm', 'beta1_pow_acc')

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None, weight_decay=None,
                 grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float()
        m = self._acc('moment', p)
        u = self._acc('inf_norm', p)
        b1p = self._acc('beta1_pow_acc', p, fill=self._b1, shape=[1])
        m.mul_(self._b1).add_(g, alpha=1 - self._b1)
        torch.maximum(u * self._b2, g.abs() + self._eps, out=u)
        pv = p._t.data.float() - (lr / (1 - b1p)) * m / u
        p._t.data.copy_(pv.to(p._t.dtype))
        b1p.mul_(self._b1)


class Adagrad(Optimizer):
    _acc_names = ('moment',)

    def __init__(self, learning_rate, epsilon=1e-6, parameters=None, weight_decay=None, grad_clip=None, name=None,
                 initial_accumulator_value=0.0):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._init = epsilon, initial_accumulator_value

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float()
        m = self._acc('moment', p, fill=self._init)
        m.addcmul_(g, g)
        p._t.data.copy_((p._t.data.float() - lr * g / (m.sqrt() + self._eps)).to(p._t.dtype))


class Adadelta(Optimizer):
    _acc_names = ('avg_squared_grad', 'avg_squared_update')

    def __init__(self, learning_rate=0.001, epsilon=1.0e-6, rho=0.95, parameters=None, weight_decay=None,
                 grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._rho = epsilon, rho

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float()
        sg = self._acc('avg_squared_grad', p)
        su = self._acc('avg_squared_update', p)
        sg.mul_(self._rho).addcmul_(g, g, value=1 - self._rho)
        upd = -torch.sqrt((su + self._eps) / (sg + self._eps)) * g
        su.mul_(self._rho).addcmul_(upd, upd, value=1 - self._rho)
        p._t.data.copy_((p._t.data.float() + lr * upd).to(p._t.dtype))


class RMSProp(Optimizer):
    _acc_names = ('momentum', 'mean_square', 'mean_grad')

    def __init__(self, learning_rate, rho=0.95, epsilon=1.0e-6, momentum=0.0, centered=False, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._rho, self._eps, self._mom, self._centered = rho, epsilon, momentum, centered

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float()
        ms = self._acc('mean_square', p)
        mom = self._acc('momentum', p)
        ms.mul_(self._rho).addcmul_(g, g, value=1 - self._rho)
        if self._centered:
            mg = self._acc('mean_grad', p)
            mg.mul_(self._rho).add_(g, alpha=1 - self._rho)
            denom = (ms - mg * mg + self._eps).sqrt()
        else:
            denom = (ms + self._eps).sqrt()
        mom.mul_(self._mom).add_(lr * g / denom)
        p._t.data.copy_((p._t.data.float() - mom).to(p._t.dtype))


class Lamb(Optimizer):
    _acc_names = ('moment1', 'moment2', 'beta1_pow_acc', 'beta2_pow_acc')

    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, multi_precision=False,
                 always_adapt=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name)
        self._wd, self._b1, self._b2, self._eps = lamb_weight_decay, beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn
        self._always_adapt = always_adapt
        self._multi_precision = multi_precision

    def _update_param(self, p, g, lr, group):
        g = g.float()
        m1, m2 = self._acc('moment1', p), self._acc('moment2', p)
        b1p = self._acc('beta1_pow_acc', p, fill=self._b1, shape=[1])
        b2p = self._acc('beta2_pow_acc', p, fill=self._b2, shape=[1])
        master = self._master(p)
        pv = master if master is not None else p._t.data.float()
        m1.mul_(self._b1).add_(g, alpha=1 - self._b1)
        m2.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
        mh = m1 / (1 - b1p)
        vh = m2 / (1 - b2p)
        wd = 0.0 if (self._exclude is not None and self._exclude(p)) else self._wd
        r = mh / (vh.sqrt() + self._eps) + wd * pv
        pn, rn = pv.norm(), r.norm()
        trust = torch.where((pn > 0) & (rn > 0), pn / rn, torch.ones_like(pn))
        _write_back(p, pv - lr * trust * r, master)
        b1p.mul_(self._b1)
        b2p.mul_(self._b2)


class NAdam(Optimizer):
    _acc_names = ('moment1', 'moment2', 'mu_product')

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1.0e-8, momentum_decay=0.004,
                 parameters=None, weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps, self._md = beta1, beta2, epsilon, momentum_decay
        self._t = {}

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float()
        t = self._t.get(p.name, 0) + 1
        self._t[p.name] = t
        m1, m2 = self._acc('moment1', p), self._acc('moment2', p)
        mu_prod = self._acc('mu_product', p, fill=1.0, shape=[1])
        mu = self._b1 * (1 - 0.5 * 0.96 ** (t * self._md))
        mu_next = self._b1 * (1 - 0.5 * 0.96 ** ((t + 1) * self._md))
        mu_prod.mul_(mu)
        m1.mul_(self._b1).add_(g, alpha=1 - self._b1)
        m2.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
        denom = (m2 / (1 - self._b2 ** t)).sqrt() + self._eps
        pv = p._t.data.float()
        pv = pv - lr * (1 - mu) / (1 - mu_prod) * g / denom - lr * mu_next / (1 - mu_prod * mu_next) * m1 / denom
        p._t.data.copy_(pv.to(p._t.dtype))


class RAdam(Optimizer):
    _acc_names = ('moment1', 'moment2')

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1.0e-8, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon
        self._t = {}

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float()
        t = self._t.get(p.name, 0) + 1
        self._t[p.name] = t
        m1, m2 = self._acc('moment1', p), self._acc('moment2', p)
        m1.mul_(self._b1).add_(g, alpha=1 - self._b1)
        m2.mul_(self._b2).addcmul_(g, g, value=1 - self._b2)
        mh = m1 / (1 - self._b1 ** t)
        rho_inf = 2 / (1 - self._b2) - 1
        rho = rho_inf - 2 * t * self._b2 ** t / (1 - self._b2 ** t)
        pv = p._t.data.float()
        if rho > 5:
            l = math.sqrt((1 - self._b2 ** t)) / (m2.sqrt() + self._eps)
            r = math.sqrt((rho - 4) * (rho - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho))
            pv = pv - lr * mh * r * l
        else:
            pv = pv - lr * mh
        p._t.data.copy_(pv.to(p._t.dtype))


class ASGD(Optimizer):
    _acc_names = ('d', 'y', 'n')

    def __init__(self, learning_rate=0.001, batch_num=1, parameters=None, weight_decay=None, grad_clip=None,
                 multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._batch_num = batch_num
        self._ys = {}
        self._step_i = {}

    def _update_param(self, p, g, lr, group):
        g = self._apply_regularization(p, g, group).float()
        d = self._acc('d', p)
        n = self._acc('n', p, shape=[1])
        i = self._step_i.get(p.name, 0)
        ys = self._ys.setdefault(p.name, [torch.zeros_like(d) for _ in range(self._batch_num)])
        idx = i % self._batch_num
        d.sub_(ys[idx]).add_(g)
        ys[idx] = g.clone()
        n.fill_(min(i + 1, self._batch_num))
        self._step_i[p.name] = i + 1
        p._t.data.copy_((p._t.data.float() - lr * d / n).to(p._t.dtype))


class Rprop(Optimizer):
    _acc_names = ('prev', 'learning_rate')

    def __init__(self, learning_rate=0.001, learning_rate_range=(1e-5, 50), parameters=None, etas=(0.5, 1.2),
                 grad_clip=None, multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name)
        self._range, self._etas = learning_rate_range, etas

    def _update_param(self, p, g, lr, group):
        g = g.float()
        prev = self._acc('prev', p)
        lrs = self._acc('learning_rate', p, fill=lr)
        sign = g * prev
        lrs.copy_(torch.where(sign > 0, lrs * self._etas[1], torch.where(sign < 0, lrs * self._etas[0], lrs)))
        lrs.clamp_(self._range[0], self._range[1])
        g = torch.where(sign < 0, torch.zeros_like(g), g)
        p._t.data.copy_((p._t.data.float() - lrs * torch.sign(g)).to(p._t.dtype))
        prev.copy_(g)


class LBFGS(Optimizer):
    def __init__(self, learning_rate=1.0, max_iter=20, max_eval=None, tolerance_grad=1e-7, tolerance_change=1e-9,
                 history_size=100, line_search_fn=None, parameters=None, weight_decay=None, grad_clip=None,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._torch_opt = torch.optim.LBFGS([p._t for p in self._parameter_list], lr=learning_rate,
                                            max_iter=max_iter, max_eval=max_eval, tolerance_grad=tolerance_grad,
                                            tolerance_change=tolerance_change, history_size=history_size,
                                            line_search_fn=line_search_fn)

    def step(self, closure=None):
        def c():
            with torch.enable_grad():
                loss = closure()
            return _unwrap(loss)
        r = self._torch_opt.step(c)
        return _wrap(r) if isinstance(r, torch.Tensor) else r
