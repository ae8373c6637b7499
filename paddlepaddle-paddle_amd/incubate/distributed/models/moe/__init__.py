"""Mixture of Experts with expert parallelism (reference: python/paddle/incubate/distributed/
models/moe/{moe_layer.py MoELayer:263, gate/{naive,gshard,switch}_gate.py, grad_clip.py}).

Dispatch on MI355X: tokens are sorted by destination expert on the device (one argsort), the
per-expert counts are exchanged with one small all-to-all, and the tokens themselves move with
one ``all_to_all_single`` over the expert-parallel group (RCCL over xGMI; every rank pair is one
direct link on an 8-GPU node).  Each rank runs its local experts on contiguous segments, then
the reverse all-to-all returns outputs which are combined with the gate weights by one
``index_add``.  The exchange is an autograd Function whose backward is the reverse exchange.

Expert compute: when the experts are homogeneous two-layer FFNs (same class, one Linear d -> f and
one Linear f -> d, an elementwise activation between them — the ExpertLayer form of the reference's
MoE tests and PaddleNLP), the local experts run as TWO batched GEMM launches over all experts
(ops/matmul.py: [E, capacity, d] @ [E, d, f], blockIdx.y = expert) instead of a Python loop of
per-expert Linears (reference kernel: paddle/phi/kernels/fusion/cutlass/moe_kernel.cu).  The
structure is verified once numerically against expert 0's own forward (activation identified
among relu / gelu / gelu-tanh / silu); anything else keeps the per-expert loop.
"""
import math

import torch
import torch.distributed as dist
import torch.nn.functional as TF

from .....nn.layer.layers import Layer
from .....nn import Linear, LayerList
from .....core.tensor import Tensor, _wrap, _unwrap
from .....nn.clip import ClipGradByGlobalNorm


def _pg(group):
    return getattr(group, 'pg', group)


def _world(group):
    if group is None or not dist.is_initialized():
        return 1, 0
    pg = _pg(group)
    return dist.get_world_size(pg), dist.get_rank(pg)


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_splits, in_splits, group):
        ctx.splits = (out_splits, in_splits)
        ctx.group = group
        out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
        _a2a_single(out, x.contiguous(), out_splits, in_splits, group)
        return out

    @staticmethod
    def backward(ctx, g):
        out_splits, in_splits = ctx.splits
        gin = g.new_empty((sum(in_splits),) + tuple(g.shape[1:]))
        _a2a_single(gin, g.contiguous(), in_splits, out_splits, ctx.group)
        return gin, None, None, None


def _a2a_single(out, inp, out_splits, in_splits, group):
    pg = _pg(group)
    if dist.get_backend(pg) != 'gloo':
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=pg)
        return
    ins = list(inp.split(in_splits, 0))
    outs = list(out.split(out_splits, 0))
    from .....distributed.communication import all_to_all_tensors
    tmp = [torch.empty_like(o) for o in outs]
    all_to_all_tensors(tmp, [i.contiguous() for i in ins], pg)
    for o, t in zip(outs, tmp):
        o.copy_(t)


# ----------------------------------------------------------------- gates
class BaseGate(Layer):
    def __init__(self, num_expert, world_size):
        super().__init__()
        self.world_size = world_size
        self.num_expert = num_expert
        self.tot_expert = world_size * num_expert
        self.loss = None

    def set_loss(self, loss):
        self.loss = loss

    def get_loss(self, clear=True):
        loss = self.loss
        if clear:
            self.loss = None
        return loss


class NaiveGate(BaseGate):
    def __init__(self, d_model, num_expert, world_size, topk=2):
        super().__init__(num_expert, world_size)
        self.gate = Linear(d_model, self.tot_expert)
        self.top_k = topk

    def forward(self, inp, return_all_scores=False):
        logits = _unwrap(self.gate(inp))
        val, idx = torch.topk(logits, self.top_k, dim=-1)
        score = torch.softmax(val, -1)
        if return_all_scores:
            return _wrap(score), _wrap(idx), _wrap(logits)
        return _wrap(score), _wrap(idx)


def _capacity_mask(idx, n_exp, capacity):
    """Keep at most ``capacity`` tokens per expert (in token order) → boolean keep mask."""
    flat = idx.reshape(-1)
    onehot = TF.one_hot(flat, n_exp)
    pos = torch.cumsum(onehot, 0) * onehot
    return (pos.sum(-1) <= capacity).reshape(idx.shape)


class GShardGate(NaiveGate):
    """Top-2 with expert capacity and the GShard load-balancing loss."""

    def __init__(self, d_model, num_expert, world_size, topk=2, capacity=(1.2, 2.4), random_routing=True,
                 group=None):
        super().__init__(d_model, num_expert, world_size, topk)
        self.capacity = capacity
        self.random_routing = random_routing

    def forward(self, x):
        score, idx, logits = super().forward(x, return_all_scores=True)
        s, i, lg = _unwrap(score), _unwrap(idx), _unwrap(logits)
        probs = torch.softmax(lg, -1)
        me = probs.mean(0)
        ce = TF.one_hot(i[:, 0], self.tot_expert).float().mean(0)
        self.set_loss(_wrap((me * ce).sum() * self.tot_expert))
        cap_rate = self.capacity[0 if self.training else 1]
        cap = int(math.ceil(cap_rate * x.shape[0] / self.tot_expert) * self.top_k)
        keep = _capacity_mask(i, self.tot_expert, cap)
        if self.random_routing and self.top_k >= 2:
            keep[:, 1] &= (2 * s[:, 1] > torch.rand_like(s[:, 1]))
        i = torch.where(keep, i, torch.full_like(i, -1))
        return _wrap(s), _wrap(i)


class SwitchGate(NaiveGate):
    """Top-1 with capacity, multiplicative jitter in training and the Switch balance loss."""

    def __init__(self, d_model, num_expert, world_size, topk=1, switch_eps=0.1, capacity=(1.2, 2.4), group=None):
        super().__init__(d_model, num_expert, world_size, 1)
        self.switch_eps = switch_eps
        self.capacity = capacity

    def forward(self, inp):
        t = _unwrap(inp)
        if self.training:
            t = t * torch.empty_like(t).uniform_(1 - self.switch_eps, 1 + self.switch_eps)
        lg = _unwrap(self.gate(_wrap(t)))
        probs = torch.softmax(lg.float(), -1)
        s, i = probs.max(-1, keepdim=True)
        cap_rate = self.capacity[0 if self.training else 1]
        cap = int(math.ceil(cap_rate * t.shape[0] / self.tot_expert))
        keep = _capacity_mask(i, self.tot_expert, cap)
        i = torch.where(keep, i, torch.full_like(i, -1))
        frac = TF.one_hot(i.clamp(min=0).reshape(-1), self.tot_expert).float().mean(0)
        self.set_loss(_wrap((frac * probs.mean(0)).sum() * self.tot_expert))
        return _wrap(s.to(lg.dtype)), _wrap(i)


# ----------------------------------------------------------------- grouped experts
_ACTS = {
    'relu': torch.relu,
    'gelu': lambda t: TF.gelu(t),
    'gelu_tanh': lambda t: TF.gelu(t, approximate='tanh'),
    'silu': TF.silu,
}


# sublayers an expert may hold besides its two Linears: parameterless, deterministic and
# mode-independent (a Dropout — or any unknown layer — keeps the expert on the per-expert loop, since
# the one-off numeric probe cannot see train/eval-dependent behaviour)
_PASSIVE = ('ReLU', 'GELU', 'Silu', 'SiLU', 'Swish', 'Sequential', 'LayerList')


def _ffn_linears(expert):
    lins = []
    for l in expert.sublayers():
        if isinstance(l, Linear):
            lins.append(l)
        elif type(l).__name__ not in _PASSIVE:
            return None
    if len(lins) != 2 or len(expert.parameters()) != sum(len(l.parameters()) for l in lins):
        return None
    return lins


def _detect_grouped(experts, d_model):
    """(order, act) when every expert is x -> lin2(act(lin1(x))) with matching shapes, else None.
    Verified numerically on expert 0 with a random probe (fp32, on the experts' device)."""
    e0 = experts[0]
    lins = _ffn_linears(e0)
    if lins is None or any(type(e) is not type(e0) for e in experts):
        return None
    a, b = lins
    if a.weight.shape[0] != d_model:
        a, b = b, a
    if a.weight.shape[0] != d_model or b.weight.shape[1] != d_model or a.weight.shape[1] != b.weight.shape[0]:
        return None
    for e in experts[1:]:
        l2 = _ffn_linears(e)
        if l2 is None or sorted(tuple(l.weight.shape) for l in l2) != sorted((tuple(a.weight.shape),
                                                                              tuple(b.weight.shape))):
            return None
    first = 0 if lins[0] is a else 1
    w = a.weight._t
    g = torch.Generator(device=w.device).manual_seed(0)
    probe = torch.randn(4, d_model, generator=g, device=w.device).to(w.dtype)
    with torch.no_grad():
        ref = _unwrap(e0(_wrap(probe))).float()
        h = probe.float() @ a.weight._t.float() + (a.bias._t.float() if a.bias is not None else 0.0)
        for name, fn in _ACTS.items():
            out = fn(h).to(w.dtype).float() @ b.weight._t.float() + (b.bias._t.float() if b.bias is not None else 0.0)
            tol = 1e-4 if w.dtype == torch.float32 else 3e-2
            if torch.allclose(out, ref, atol=tol * (ref.abs().max().item() + 1e-3), rtol=tol):
                return first, name
    return None


def _grouped_ffn(experts, spec, per_exp, d_model):
    """All experts' FFNs as two batched GEMMs over a [E, cap, d] zero-padded token block."""
    counts = [c.shape[0] for c in per_exp]
    cap = -(-max(max(counts), 1) // 8) * 8  # the GEMM's row contract
    x = per_exp[0]
    rows = torch.cat([torch.arange(c, device=x.device) + j * cap for j, c in enumerate(counts)])
    flat = _grouped_ffn_rows(experts, spec, torch.cat(per_exp, 0), rows, cap, d_model)
    return list(flat.split(counts, 0))


def _ep_regroup_index(rc, E, cap, device):
    """Expert-parallel regroup as ONE index: row i of the all-to-all receive buffer (grouped by
    source rank, then local expert; rc[r][j] rows each) goes to slot j * cap + (rows of expert j
    from ranks < r) + its position inside its segment of the [E, cap] expert-major block.  The
    same index maps the block's outputs back to receive order (the return all-to-all's layout),
    so neither direction loops over (rank, expert) pieces."""
    W = len(rc)
    seg_len = [rc[r][j] for r in range(W) for j in range(E)]
    n = sum(seg_len)
    seg_start, acc = [], 0
    for c in seg_len:
        seg_start.append(acc)
        acc += c
    base, run = [], [0] * E
    for r in range(W):
        for j in range(E):
            base.append(j * cap + run[j])
            run[j] += rc[r][j]
    lens = torch.tensor(seg_len, device=device)
    seg = torch.repeat_interleave(torch.arange(W * E, device=device), lens, output_size=n)
    local = torch.arange(n, device=device) - torch.tensor(seg_start, device=device)[seg]
    return torch.tensor(base, device=device)[seg] + local


def _grouped_ffn_rows(experts, spec, x_rows, dst, cap, d_model):
    """Two batched GEMMs over the [E, cap, d] block filled by ``x_rows`` at slots ``dst``; returns
    the output rows in the order of ``x_rows``."""
    from ..... import ops
    first, act = spec
    E = len(experts)
    lins = [_ffn_linears(e) for e in experts]
    l1 = [l[first] for l in lins]
    l2 = [l[1 - first] for l in lins]
    blk = x_rows.new_zeros(E * cap, d_model).index_copy(0, dst, x_rows).view(E, cap, d_model)
    w1 = torch.stack([l.weight._t for l in l1])  # [E, d, f]
    w2 = torch.stack([l.weight._t for l in l2])  # [E, f, d]
    h = ops.matmul.matmul(blk, w1)
    if l1[0].bias is not None:
        h = h + torch.stack([l.bias._t for l in l1]).unsqueeze(1)
    h = _ACTS[act](h)
    y = ops.matmul.matmul(h, w2)
    if l2[0].bias is not None:
        y = y + torch.stack([l.bias._t for l in l2]).unsqueeze(1)
    return y.reshape(E * cap, -1).index_select(0, dst)


# ----------------------------------------------------------------- layer
class MoELayer(Layer):
    def __init__(self, d_model, experts, gate=None, moe_group=None, mp_group=None, recompute_interval=0,
                 recompute_ctx=None):
        super().__init__()
        self.group = moe_group
        self.world_size, self.rank = _world(moe_group)
        self.experts = experts if isinstance(experts, LayerList) else LayerList(list(experts))
        self.num_expert = len(self.experts)
        self.d_model = d_model
        self.recompute_interval = recompute_interval
        gate = gate if gate is not None else {}
        if isinstance(gate, dict):
            typ = gate.get('type', 'gshard')
            topk = gate.get('top_k', 2)
            if typ == 'naive':
                gate = NaiveGate(d_model, self.num_expert, self.world_size, topk)
            elif typ == 'gshard':
                gate = GShardGate(d_model, self.num_expert, self.world_size, topk, group=moe_group)
            elif typ == 'switch':
                gate = SwitchGate(d_model, self.num_expert, self.world_size, group=moe_group)
            else:
                raise ValueError(f"unknown gate type {typ}")
        self.gate = gate
        self.top_k = getattr(gate, 'top_k', 1)
        self._grouped = {}  # training flag -> (order, act) once verified, or False (per-expert loop)

    def forward(self, inp):
        t = _unwrap(inp)
        shape = t.shape
        x = t.reshape(-1, shape[-1])
        score, idx = self.gate(_wrap(x))
        s, e = _unwrap(score), _unwrap(idx)             # [T, k]
        T, k = e.shape
        tok = torch.arange(T, device=x.device).repeat_interleave(k)
        ef, sf = e.reshape(-1), s.reshape(-1)
        valid = ef >= 0
        tok, ef, sf = tok[valid], ef[valid], sf[valid]
        order = torch.argsort(ef, stable=True)
        tok, ef, sf = tok[order], ef[order], sf[order]
        tot = self.num_expert * self.world_size
        counts = torch.bincount(ef, minlength=tot)            # tokens this rank sends to each global expert
        send = x.index_select(0, tok)
        if self.world_size > 1:
            recv_counts = torch.empty_like(counts)
            _a2a_single(recv_counts, counts, [self.num_expert] * self.world_size,
                        [self.num_expert] * self.world_size, self.group)
            in_splits = counts.view(self.world_size, self.num_expert).sum(1).tolist()
            out_splits = recv_counts.view(self.world_size, self.num_expert).sum(1).tolist()
            recv = _AllToAll.apply(send, out_splits, in_splits, self.group)
        mode = bool(self.training)
        if mode not in self._grouped:  # probed per mode: train/eval behaviour may differ
            self._grouped[mode] = _detect_grouped(list(self.experts), self.d_model) or False
        spec = self._grouped[mode]
        if self.world_size > 1 and spec and self.num_expert > 1:
            # grouped experts: the receive buffer goes straight into the expert-major block and the
            # block's outputs straight back into receive order (one index each way)
            rc = recv_counts.view(self.world_size, self.num_expert).tolist()
            cap = -(-max(max(sum(rc[r][j] for r in range(self.world_size)) for j in range(self.num_expert)), 1)
                    // 8) * 8
            dst = _ep_regroup_index(rc, self.num_expert, cap, recv.device)
            back_in = _grouped_ffn_rows(list(self.experts), spec, recv, dst, cap, self.d_model)
            ret = _AllToAll.apply(back_in, in_splits, out_splits, self.group)
            y = torch.zeros(T, ret.shape[-1], dtype=ret.dtype, device=ret.device)
            y = y.index_add(0, tok, ret * sf.unsqueeze(-1).to(ret.dtype))
            return _wrap(y.reshape(shape[:-1] + (ret.shape[-1],)))
        if self.world_size > 1:
            # recv is grouped by source rank, then local expert; regroup by local expert
            rc = recv_counts.view(self.world_size, self.num_expert)
            seg = list(recv.split(rc.reshape(-1).tolist(), 0))
            per_exp = [torch.cat([seg[r * self.num_expert + j] for r in range(self.world_size)], 0)
                       for j in range(self.num_expert)]
        else:
            per_exp = list(send.split(counts.tolist(), 0))
        if spec and self.num_expert > 1:
            outs = _grouped_ffn(list(self.experts), spec, per_exp, self.d_model)
        else:
            outs = []
            for j, chunk in enumerate(per_exp):
                if chunk.shape[0] == 0:
                    outs.append(chunk.new_zeros((0, self.d_model)))
                    continue
                outs.append(_unwrap(self.experts[j](_wrap(chunk))))
        if self.world_size > 1:
            rc = recv_counts.view(self.world_size, self.num_expert)
            pieces = [o.split(rc[:, j].tolist(), 0) for j, o in enumerate(outs)]
            back_in = torch.cat([pieces[j][r] for r in range(self.world_size) for j in range(self.num_expert)], 0)
            ret = _AllToAll.apply(back_in, in_splits, out_splits, self.group)
        else:
            ret = torch.cat(outs, 0) if outs else send
        y = torch.zeros(T, ret.shape[-1], dtype=ret.dtype, device=ret.device)
        y = y.index_add(0, tok, ret * sf.unsqueeze(-1).to(ret.dtype))
        return _wrap(y.reshape(shape[:-1] + (ret.shape[-1],)))


class ClipGradForMOEByGlobalNorm(ClipGradByGlobalNorm):
    """Global-norm clip where expert parameters' squared norms are summed across the MoE group
    (they are distinct on each rank) and shared parameters are counted once."""

    def __init__(self, clip_norm, is_expert_param_func=None, moe_group=None, group_name="default_moe_group"):
        super().__init__(clip_norm)
        self.is_expert_param_func = is_expert_param_func
        self.moe_group = moe_group

    def __call__(self, params_grads):
        if self.moe_group is None or not dist.is_initialized() or self.is_expert_param_func is None:
            return super().__call__(params_grads)
        exp_sq = torch.zeros((), device=_unwrap(params_grads[0][0]).device)
        norm_sq = torch.zeros_like(exp_sq)
        for p, g in params_grads:
            if g is None:
                continue
            s = _unwrap(g).float().pow(2).sum()
            if self.is_expert_param_func(p):
                exp_sq = exp_sq + s
            else:
                norm_sq = norm_sq + s
        dist.all_reduce(exp_sq, group=_pg(self.moe_group))
        total = torch.sqrt(exp_sq + norm_sq)
        scale = torch.clamp(self.clip_norm / torch.clamp(total, min=self.clip_norm), max=1.0)
        out = []
        for p, g in params_grads:
            if g is not None:
                _unwrap(g).mul_(scale.to(_unwrap(g).dtype))
            out.append((p, g))
        return out


ClipGradByGlobalNorm = ClipGradForMOEByGlobalNorm
_ = Tensor
