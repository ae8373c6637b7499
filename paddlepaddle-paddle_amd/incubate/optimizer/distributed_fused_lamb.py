"""DistributedFusedLamb (reference: python/paddle/incubate/optimizer/distributed_fused_lamb.py:115,
kernel paddle/phi/kernels/fusion/gpu/distributed_fused_lamb_kernel.cu).

LAMB over ALL parameters as multi-tensor (``torch._foreach_*``) launches on fp32 master copies —
one launch per elementwise stage for the whole model instead of a kernel chain per parameter, the
per-parameter trust ratios from two multi-tensor norm launches — with the reference's distributed
semantics: gradients are all-reduced over the data-parallel world (RCCL) before the update, one
flat all-reduce per dtype (summed when ``is_grad_scaled_by_nranks``, else averaged), global-norm
clipping before or after that all-reduce (``clip_after_allreduce``), ``exclude_from_weight_decay_fn``
and ``gradient_accumulation_steps`` (gradients accumulate in fp32 across ``step()`` calls; the
update runs every N-th call).
"""
import torch
import torch.distributed as dist

from ...core.tensor import _unwrap
from ...optimizer.optimizer import Optimizer
from ...nn.clip import ClipGradByGlobalNorm


class DistributedFusedLamb(Optimizer):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, clip_after_allreduce=True,
                 is_grad_scaled_by_nranks=True, alignment=128, use_master_param_norm=True,
                 gradient_accumulation_steps=1, use_master_acc_grad=True, nproc_per_node=None,
                 use_hierarchical_allreduce=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name)
        if grad_clip is not None and not isinstance(grad_clip, ClipGradByGlobalNorm):
            raise TypeError("DistributedFusedLamb only supports ClipGradByGlobalNorm")
        self._wd, self._b1, self._b2, self._eps = float(lamb_weight_decay), float(beta1), float(beta2), float(epsilon)
        self._exclude = exclude_from_weight_decay_fn
        self._clip_after = bool(clip_after_allreduce)
        self._scaled_by_nranks = bool(is_grad_scaled_by_nranks)
        self._acc_steps = max(1, int(gradient_accumulation_steps))
        self._use_master_norm = bool(use_master_param_norm)
        self._calls = 0
        self._state = None

    def _build(self):
        ps = [p for p in self._parameter_list if p.trainable]
        master = [p._t.detach().float().clone() for p in ps]
        self._state = {
            'params': ps,
            'master': master,
            'm': [torch.zeros_like(x) for x in master],
            'v': [torch.zeros_like(x) for x in master],
            'acc': [torch.zeros_like(x) for x in master] if self._acc_steps > 1 else None,
            'wd': [0.0 if (self._exclude is not None and self._exclude(p)) else self._wd for p in ps],
            'step': 0,
        }

    def _allreduce(self, grads):
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1 or not grads:
            return
        world = dist.get_world_size()
        by_dt = {}
        for g in grads:
            by_dt.setdefault((g.dtype, g.device), []).append(g)
        for gs in by_dt.values():
            flat = torch.cat([g.reshape(-1) for g in gs])
            dist.all_reduce(flat)
            if not self._scaled_by_nranks:
                flat.div_(world)
            off = 0
            for g in gs:
                n = g.numel()
                g.copy_(flat[off:off + n].view_as(g))
                off += n

    def _clip_scale(self, grads):
        clip = self._grad_clip
        if clip is None or not grads:
            return None
        norms = torch._foreach_norm(grads)
        total = torch.stack([n.float() for n in norms]).pow(2).sum().sqrt()
        return torch.clamp(clip.clip_norm / torch.clamp(total, min=clip.clip_norm), max=1.0)

    @torch.no_grad()
    def step(self):
        if self._state is None:
            self._build()
        st = self._state
        ps = st['params']
        live = [(i, p._t.grad) for i, p in enumerate(ps) if p._t.grad is not None]
        if not live:
            return
        idx = [i for i, _ in live]
        grads = [g.float() if g.dtype != torch.float32 else g.clone() for _, g in live]
        self._calls += 1
        if st['acc'] is not None:
            accs = [st['acc'][i] for i in idx]
            torch._foreach_add_(accs, grads)
            if self._calls % self._acc_steps:
                return
            grads = [a / self._acc_steps for a in accs]
            for a in accs:
                a.zero_()
        if not self._clip_after:
            s = self._clip_scale(grads)
            if s is not None:
                torch._foreach_mul_(grads, s)
        self._allreduce(grads)
        if self._clip_after:
            s = self._clip_scale(grads)
            if s is not None:
                torch._foreach_mul_(grads, s)
        st['step'] += 1
        t = st['step']
        b1, b2 = self._b1, self._b2
        ms = [st['m'][i] for i in idx]
        vs = [st['v'][i] for i in idx]
        ws = [st['master'][i] for i in idx]
        torch._foreach_mul_(ms, b1)
        torch._foreach_add_(ms, grads, alpha=1 - b1)
        torch._foreach_mul_(vs, b2)
        torch._foreach_addcmul_(vs, grads, grads, value=1 - b2)
        bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
        mh = torch._foreach_div(ms, bc1)
        den = torch._foreach_sqrt(torch._foreach_div(vs, bc2))
        torch._foreach_add_(den, self._eps)
        r = torch._foreach_div(mh, den)
        wds = [st['wd'][i] for i in idx]
        for rr, w, wd in zip(r, ws, wds):
            if wd:
                rr.add_(w, alpha=wd)
        pn = torch._foreach_norm(ws if self._use_master_norm else [ps[i]._t.float() for i in idx])
        rn = torch._foreach_norm(r)
        lr = self.get_lr()
        for rr, w, a, b, i in zip(r, ws, pn, rn, idx):
            trust = torch.where((a > 0) & (b > 0), a / b, torch.ones_like(a))
            w.sub_(rr * (lr * trust))
            ps[i]._t.data.copy_(w.to(ps[i]._t.dtype))
        self._global_step += 1

    def state_dict(self):
        sd = super().state_dict()
        if self._state is not None:
            st = self._state
            for p, m, v, w in zip(st['params'], st['m'], st['v'], st['master']):
                sd[f"{p.name}_moment1_0"] = m
                sd[f"{p.name}_moment2_0"] = v
                sd[f"{p.name}_fp32_master_0"] = w
            sd['@lamb_step@'] = st['step']
        return sd

    def set_state_dict(self, state_dict):
        if self._state is None:
            self._build()
        st = self._state
        for p, m, v, w in zip(st['params'], st['m'], st['v'], st['master']):
            for key, buf in ((f"{p.name}_moment1_0", m), (f"{p.name}_moment2_0", v), (f"{p.name}_fp32_master_0", w)):
                if key in state_dict:
                    val = state_dict[key]
                    buf.copy_(_unwrap(val) if not isinstance(val, torch.Tensor) else val)
        st['step'] = int(state_dict.get('@lamb_step@', st['step']))
