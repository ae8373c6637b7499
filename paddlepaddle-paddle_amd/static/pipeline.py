"""Static-graph pipeline parallelism (reference: python/paddle/distributed/fleet/meta_optimizers/
pipeline_optimizer.py + the section/1F1B program runners: the program is split by the device of
each op — ``static.device_guard('gpu:N')`` — into one section per pipeline stage, activations
cross stages with send_v2 / recv_v2, and ``accumulate_steps`` micro-batches run per step).

Here the recorded program is not rewritten: every rank holds the whole op list and executes only
the nodes of its own stage (``Node.meta['stage']``; nodes outside any guard belong to the stage
of the previous guarded node, or stage 0).  Boundary values — produced on a stage < b and read on
a stage >= b — are sent from stage b-1 to stage b (values skipping a stage are forwarded), each
preceded by a small shape/dtype header.  Schedule (``schedule_mode``):
  * FThenB: all micro-batch forwards, then all backwards (reverse stage order);
  * 1F1B: warm-up forwards (stages - stage - 1), then one-forward-one-backward, then cool-down —
    at most ``stages`` micro-batches of activations alive per stage;
  * ZBH1: 1F1B's order with every backward split into B (input gradients, sent upstream at once)
    and W (weight gradients, deferred by SplitBwLinear and run behind the send).
Backward: the last stage runs loss/acc backward; every other stage receives the gradients of the
values it sent and continues autograd from them; gradients of the values it received go back.
After the last micro-batch the data-parallel all-reduce, the optimizer step and clear_grad run
(the StaticMinimize policy of the minimize node).  The mean micro-batch loss is broadcast over
the pipe group so every stage can fetch it.
"""
import torch
import torch.distributed as dist

from .program import Ref

_DT = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32, torch.bool, torch.float64,
       torch.uint8, torch.int8]


class PipelineConfig:
    """One rank's view of a static pipeline.  ``vpp`` > 1 (schedule 'VPP'): the program's
    device_guard stages are S * vpp chunks, chunk c on pipe rank c % S, run in the interleaved
    1F1B order; gradients then travel on ``grad_group`` (a second communicator over the same
    ranks), so every (src, dst) channel carries one kind of message in one order."""

    def __init__(self, stage, nstages, acc, group, prev_rank, next_rank, schedule='1F1B', vpp=1, grad_group=None):
        self.stage, self.nstages, self.acc = stage, nstages, max(1, int(acc))
        self.group, self.prev, self.next = group, prev_rank, next_rank
        self.schedule = schedule
        self.vpp = max(1, int(vpp or 1))
        self.grad_group = grad_group


def _stages(nodes, nstages):
    out, cur = [], 0
    for n in nodes:
        s = n.meta.get('stage') if n.meta else None
        if s is not None:
            cur = max(0, min(int(s), nstages - 1))
        out.append(cur)
    return out


def _refs(obj, acc):
    if isinstance(obj, Ref):
        acc.add(obj.vid)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _refs(o, acc)
    elif isinstance(obj, dict):
        for o in obj.values():
            _refs(o, acc)
    elif isinstance(obj, slice):
        _refs([obj.start, obj.stop, obj.step], acc)


def _outs(o, acc):
    if o is None:
        return
    if isinstance(o, int):
        acc.add(o)
    else:
        for x in o:
            _outs(x, acc)


class _Plan:
    """Per program and stage count: the node list of each stage and the boundary value sets."""

    def __init__(self, prog, nstages):
        body = [n for n in prog.nodes if n.kind != 'minimize']
        st = _stages(body, nstages)
        self.nodes = [[n for n, s in zip(body, st) if s == k] for k in range(nstages)]
        produced_at, used_at = {}, {}
        for n, s in zip(body, st):
            ins = set()
            _refs(n.args, ins)
            _refs(n.kwargs, ins)
            for v in ins:
                used_at.setdefault(v, set()).add(s)
            outs = set()
            _outs(n.outs, outs)
            for v in outs:
                produced_at[v] = s
        mn = [n for n in prog.nodes if n.kind == 'minimize']
        self.loss_vid = mn[-1].args[0].vid if mn else None
        if self.loss_vid is not None:
            used_at.setdefault(self.loss_vid, set()).add(nstages - 1)
        # X[b]: values crossing boundary b (stage b-1 -> b), sorted for a deterministic wire order
        self.cross = [[] for _ in range(nstages + 1)]
        for v, ps in produced_at.items():
            last = max(used_at.get(v, {ps}))
            for b in range(ps + 1, last + 1):
                self.cross[b].append(v)
        for b in range(nstages + 1):
            self.cross[b].sort()


def _plan(prog, nstages):
    key = ('_pp_plan', nstages, len(prog.nodes))
    p = getattr(prog, '_pp_plan_cache', None)
    if p is None or p[0] != key:
        p = (key, _Plan(prog, nstages))
        prog._pp_plan_cache = p
    return p[1]


def _send(t, dst, dev, works, group=None):
    """Non-blocking send (header, then data): receives are blocking and issued in program order,
    sends never wait, so the 1F1B steady state (a stage sending activations forward while its
    successor sends gradients back) cannot deadlock.  ``works`` keeps buffers alive until waited."""
    t = t.detach().to(dev).contiguous()
    hdr = torch.zeros(10, dtype=torch.int64)
    hdr[0], hdr[1] = t.dim(), _DT.index(t.dtype)
    for i, s in enumerate(t.shape):
        hdr[2 + i] = s
    hdr = hdr.to(dev)
    works.append((dist.isend(hdr, dst, group=group), hdr))
    works.append((dist.isend(t, dst, group=group), t))


def _recv(src, dev, group=None):
    hdr = torch.zeros(10, dtype=torch.int64, device=dev)
    dist.recv(hdr, src, group=group)
    nd, dt = int(hdr[0]), _DT[int(hdr[1])]
    t = torch.empty([int(x) for x in hdr[2:2 + nd]], dtype=dt, device=dev)
    dist.recv(t, src, group=group)
    return t


def _split_feed(prog, feed, acc):
    """Micro-batch feeds: every fed value with a leading batch dim divisible by acc is split."""
    parts = [dict() for _ in range(acc)]
    for name, v in (feed or {}).items():
        t = v._t if hasattr(v, '_t') else v
        if isinstance(t, torch.Tensor) or hasattr(t, 'shape'):
            tt = t if isinstance(t, torch.Tensor) else torch.as_tensor(t)
            if tt.dim() > 0 and tt.shape[0] % acc == 0:
                for i, c in enumerate(tt.chunk(acc, 0)):
                    parts[i][name] = c
                continue
        for i in range(acc):
            parts[i][name] = v
    return parts


def _found_inf_sync(pol, cfg, dev):
    """found-inf flag MAX-reduced over the pipe group (each stage checks only its own parameters)
    and the data-parallel group, so every rank of the step skips or applies the update together."""
    def sync(found):
        t = torch.tensor([1.0 if found else 0.0], device=dev)
        if cfg.group is not None and cfg.nstages > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=cfg.group.pg)
        if pol._nranks() > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=getattr(pol.dp_group, 'pg', None))
        return bool(t.item() > 0)
    return sync


def _run_vpp(prog, feed, dev, pol, cfg, run_forward, comm_dev, works):
    """Interleaved (virtual-stage) pipeline step: this rank runs chunks s, s + S, ... of the
    S * V device_guard stages (reference passes/pipeline_scheduler_pass/pipeline_vpp.py)."""
    from ..distributed.fleet.meta_parallel.zero_bubble_utils import interleaved_units
    s, S, V, acc = cfg.stage, cfg.nstages, cfg.vpp, cfg.acc
    C = S * V
    plan = _plan(prog, C)
    ranks = list(cfg.group.ranks)
    prev, nxt = ranks[(s - 1) % S], ranks[(s + 1) % S]
    apg = getattr(cfg.group, 'pg', None)
    gpg = getattr(cfg.grad_group, 'pg', None)
    feeds = _split_feed(prog, feed, acc)
    state, losses = {}, []
    amp = pol._amp()
    merge = pol.k_steps if pol.k_steps > 1 else 1
    div = float(acc * (merge if pol.avg else 1))
    for kind, v, m in interleaved_units(acc, V, S, s):
        c = v * S + s
        if kind == 'F':
            env, rv = {}, {}
            if c > 0:
                for vid in plan.cross[c]:
                    t = _recv(prev, comm_dev, apg).to(dev if dev is not None else comm_dev)
                    if t.is_floating_point():
                        t.requires_grad_(True)
                    env[vid] = t
                    rv[vid] = t
            run_forward(plan.nodes[c], env, feeds[m])
            sv = {}
            if c < C - 1:
                for vid in plan.cross[c + 1]:
                    _send(env[vid], nxt, comm_dev, works, apg)
                    sv[vid] = env[vid]
            state[(v, m)] = (env, rv, sv)
        else:
            env, rv, sv = state.pop((v, m))
            if c == C - 1:
                loss = env[plan.loss_vid]
                losses.append(loss.detach().float().reshape(-1)[0])
                if amp is not None:
                    amp._scaled_backward(loss, div)
                else:
                    (loss / div).backward()
            else:
                ts, gs = [], []
                for vid in plan.cross[c + 1]:
                    g = _recv(nxt, comm_dev, gpg)
                    t = sv[vid]
                    if t.requires_grad and t.is_floating_point():
                        ts.append(t)
                        gs.append(g.to(t.device, t.dtype))
                if ts:
                    torch.autograd.backward(ts, gs)
            if c > 0:
                for vid in plan.cross[c]:
                    t = rv[vid]
                    g = t.grad if (t.is_floating_point() and t.grad is not None) else torch.zeros_like(t)
                    _send(g, prev, comm_dev, works, gpg)
    return losses, plan


def run_pipeline(prog, feed, dev, pol, cfg, run_forward):
    """Execute one pipelined training step of ``prog`` on this rank's stage.  ``run_forward(nodes,
    env, feed)`` binds the feeds into ``env`` and interprets ``nodes`` (executor internals)."""
    if cfg.vpp > 1:
        comm_dev = dev if (dev is not None and torch.device(dev).type == 'cuda') else torch.device('cpu')
        works = []
        losses, plan = _run_vpp(prog, feed, dev, pol, cfg, run_forward, comm_dev, works)
        return _finish_step(pol, cfg, comm_dev, works, losses, plan)
    plan = _plan(prog, cfg.nstages)
    s, S, acc = cfg.stage, cfg.nstages, cfg.acc
    comm_dev = dev if (dev is not None and torch.device(dev).type == 'cuda') else torch.device('cpu')
    feeds = _split_feed(prog, feed, acc)
    envs, recvd, sent = [None] * acc, [None] * acc, [None] * acc
    losses = []
    works = []

    def forward(m):
        env = {}
        rv = {}
        if s > 0:
            for v in plan.cross[s]:
                t = _recv(cfg.prev, comm_dev).to(dev if dev is not None else comm_dev)
                if t.is_floating_point():
                    t.requires_grad_(True)
                env[v] = t
                rv[v] = t
        run_forward(plan.nodes[s], env, feeds[m])
        if s < S - 1:
            sv = {}
            for v in plan.cross[s + 1]:
                _send(env[v], cfg.next, comm_dev, works)
                sv[v] = env[v]
            sent[m] = sv
        envs[m], recvd[m] = env, rv

    amp = pol._amp()
    merge = pol.k_steps if pol.k_steps > 1 else 1
    div = float(acc * (merge if pol.avg else 1))

    def backward(m):
        env = envs[m]
        if s == S - 1:
            loss = env[plan.loss_vid]
            losses.append(loss.detach().float().reshape(-1)[0])
            if amp is not None:
                # loss scaling: the scaled gradient flows back through every stage's boundary sends
                amp._scaled_backward(loss, div)
            else:
                (loss / div).backward()
        else:
            ts, gs = [], []
            for v in plan.cross[s + 1]:
                g = _recv(cfg.next, comm_dev)
                t = sent[m][v]
                if t.requires_grad and t.is_floating_point():
                    ts.append(t)
                    gs.append(g.to(t.device, t.dtype))
            if ts:
                torch.autograd.backward(ts, gs)
        if s > 0:
            for v in plan.cross[s]:
                t = recvd[m][v]
                g = t.grad if (t.is_floating_point() and t.grad is not None) else torch.zeros_like(t)
                _send(g, cfg.prev, comm_dev, works)
        envs[m] = recvd[m] = sent[m] = None  # free this micro-batch's activations

    kind = cfg.schedule.upper()
    if kind == 'ZBH1' and amp is not None:
        kind = '1F1B'  # AMP's scaled backward keeps the whole backward together
    if kind == 'FTHENB':
        for m in range(acc):
            forward(m)
        for m in range(acc):
            backward(m)
    elif kind == 'ZBH1':
        # zero bubble (H1): 1F1B's F / B order, each backward split into B (input gradients, sent
        # upstream at once) and W (the deferred weight-gradient GEMMs of SplitBwLinear, run behind
        # the send) — reference passes/pipeline_scheduler_pass/pipeline_zero_bubble.py
        from ..distributed.fleet.meta_parallel.zero_bubble_utils import (WeightGradStore, schedule_order,
                                                                          static_substitutions)
        from . import executor as _ex
        WeightGradStore.clear()
        prev_zb, prev_active = _ex._ZB['map'], WeightGradStore.active
        _ex._ZB['map'], WeightGradStore.active = static_substitutions(), True
        try:
            for op, m in schedule_order('ZBH1', S, s, acc):
                if op == 'F':
                    forward(m)
                elif op == 'B':
                    backward(m)
                    WeightGradStore.flush()
                else:
                    WeightGradStore.pop()
        finally:
            _ex._ZB['map'], WeightGradStore.active = prev_zb, prev_active
            WeightGradStore.clear()
    else:  # 1F1B
        warm = min(acc, S - s - 1)
        for m in range(warm):
            forward(m)
        f, b = warm, 0
        while f < acc:
            forward(f)
            f += 1
            backward(b)
            b += 1
        while b < acc:
            backward(b)
            b += 1
    return _finish_step(pol, cfg, comm_dev, works, losses, plan)


def _finish_step(pol, cfg, comm_dev, works, losses, plan):
    """Wait for the sends, run the update (every k-th run under gradient merge) and broadcast the
    mean micro-batch loss of the pipe's last stage to every stage."""
    amp = pol._amp()
    merge = pol.k_steps if pol.k_steps > 1 else 1
    S = cfg.nstages
    for w, _ in works:
        w.wait()
    # the update (every k-th run under gradient merge): data-parallel reduction, then the AMP
    # unscale / finite check / skip-or-step / scale update or the plain optimizer step
    pol._micro += 1
    if pol._micro % merge == 0:
        if pol._nranks() > 1:
            pol._allreduce_grads()
        if amp is not None:
            amp._apply_update(_found_inf_sync(pol, cfg, comm_dev))
        else:
            opt = pol._plain()
            opt.step()
            opt.clear_grad()
    # mean micro-batch loss on every stage of the pipe group (src: the last stage)
    val = torch.stack(losses).mean() if losses else torch.zeros((), dtype=torch.float32)
    val = val.to(comm_dev)
    if cfg.group is not None and S > 1:
        dist.broadcast(val, cfg.group.ranks[-1], group=cfg.group.pg)
    out = {}
    if plan.loss_vid is not None:
        out[plan.loss_vid] = val
    return out
