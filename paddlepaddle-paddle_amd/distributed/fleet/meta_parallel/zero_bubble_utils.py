"""Zero-bubble pipeline scheduling (reference: python/paddle/distributed/passes/pipeline_scheduler_pass/
pipeline_zero_bubble.py:32 — ZB-H1 of "Zero Bubble Pipeline Parallelism", Qi et al.; and the
weight-gradient store of paddle/distributed/fleet/meta_parallel/zero_bubble_utils.py).

Backward is split into B (the input gradient, which the previous stage waits for) and W (the weight
gradients, which nobody waits for).  While a ``WeightGradStore`` is active, ``F.linear`` runs as
``SplitBwLinear``: its backward computes dX only and queues the dW / db GEMMs as a closure; the
pipeline schedule sends the input gradient upstream right after B and runs the micro-batch's W
behind the send, so the upstream stage's B no longer waits for this stage's weight gradients.
The F / B order is 1F1B's, so the activation memory is 1F1B's (ZB-H1).

``schedule_order(kind, S, s, M)`` gives one stage's op sequence; ``simulate`` plays the sequences of
all stages against each other (F after the previous stage's F, B after the next stage's B, W after
its own B) and reports makespan and bubble fraction — the schedule's shape, separate from the run.
"""
import collections

import torch


class WeightGradStore:
    """Deferred weight-gradient closures, grouped per micro-batch backward.  ``active``: F.linear
    records SplitBwLinear (set by a zero-bubble pipeline for its whole batch)."""
    active = False
    deferred = 0  # weight-gradient closures queued so far (diagnostics / tests)
    _cur = []
    _ready = collections.deque()

    @classmethod
    def put(cls, fn):
        cls._cur.append(fn)
        cls.deferred += 1

    @classmethod
    def flush(cls):
        """Close the current backward's group (one micro-batch's W)."""
        cls._ready.append(cls._cur)
        cls._cur = []

    @classmethod
    def pop(cls):
        """Run the oldest group of weight-gradient closures."""
        for fn in cls._ready.popleft():
            fn()

    @classmethod
    def pending(cls):
        return len(cls._ready)

    @classmethod
    def clear(cls):
        cls._cur = []
        cls._ready.clear()


def _accumulate(p, g):
    """p.grad += g (p a paddle Parameter or a torch tensor); fires p's deferred grad-ready hooks."""
    t = p._t if hasattr(p, '_t') else p
    with torch.no_grad():
        if t.grad is None:
            t.grad = g.to(t.dtype).reshape(t.shape).clone()
        else:
            t.grad.add_(g.to(t.grad.dtype).reshape(t.grad.shape))
    if hasattr(p, '__dict__') and p.__dict__.get('_grad_deferred'):
        from ....parallel.flat_buffer import complete_deferred
        complete_deferred(p)


class SplitBwLinear(torch.autograd.Function):
    """y = x @ W (+ b), W stored [in, out]; backward returns dX and queues dW, db (WeightGradStore)."""

    @staticmethod
    def forward(ctx, x, w, b, wp, bp):
        ctx.save_for_backward(x, w)
        ctx.wp, ctx.bp = wp, bp
        y = torch.matmul(x, w)
        return y + b if b is not None else y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = torch.matmul(dy, w.t()) if ctx.needs_input_grad[0] else None
        need_w, need_b = ctx.needs_input_grad[1], len(ctx.needs_input_grad) > 2 and ctx.needs_input_grad[2]
        wp, bp = ctx.wp, ctx.bp
        if need_w or need_b:
            x2 = x.reshape(-1, x.shape[-1]).detach()
            dy2 = dy.reshape(-1, dy.shape[-1]).detach()
            from ....parallel.flat_buffer import defer_grad
            if need_w:
                defer_grad(wp)
            if need_b and bp is not None:
                defer_grad(bp)

            def w_pass():
                if need_w:
                    _accumulate(wp, x2.t().matmul(dy2))
                if need_b and bp is not None:
                    _accumulate(bp, dy2.sum(0))
            WeightGradStore.put(w_pass)
        return dx, None, None, None, None


def split_linear(x, w, b, weight, bias):
    """F.linear under an active WeightGradStore: x, w, b the torch operands as computed with (an
    AMP cast of the parameter included); weight / bias the Parameters the deferred gradients
    accumulate into."""
    return SplitBwLinear.apply(x, w, b, weight, bias)


def _is_weight(t):
    return isinstance(t, torch.Tensor) and t.is_leaf and t.requires_grad and t.dim() == 2


def static_substitutions():
    """Recorded GEMM targets of a static program -> SplitBwLinear when the right operand is a
    trainable 2-D parameter (the static pipeline's zero-bubble forward; the Executor applies them
    while ``WeightGradStore.active``)."""
    def _bias(b):
        return b if isinstance(b, torch.Tensor) and b.is_leaf and b.requires_grad else None

    def addmm(b, x, w, *a, **k):
        if not a and not k and _is_weight(w) and torch.is_grad_enabled() and b.dim() == 1:
            return split_linear(x, w, b, w, _bias(b))
        return torch.addmm(b, x, w, *a, **k)

    def mm(x, w, *a, **k):
        if not a and not k and _is_weight(w) and torch.is_grad_enabled() and x.dim() == 2:
            return split_linear(x, w, None, w, None)
        return torch.mm(x, w, *a, **k)

    def matmul(x, w, *a, **k):
        if not a and not k and _is_weight(w) and torch.is_grad_enabled() and x.dim() >= 2:
            return split_linear(x, w, None, w, None)
        return torch.matmul(x, w, *a, **k)
    return {torch.addmm: addmm, torch.mm: mm, torch.matmul: matmul}


# ------------------------------------------------------------------ schedules + simulator
def schedule_order(kind, S, s, M):
    """Op sequence of stage s (of S) over M micro-batches: [('F'|'B'|'W'|'BW', i)].
    '1F1B': warm-up forwards, then one forward / one full backward ('BW': the input gradient is
    sent upstream only after the weight gradients too).
    'ZBH1': the same F / B order with each backward split: B computes and sends the input gradient,
    then W computes the weight gradients while the previous stage already runs its B.  The
    cool-down chain of B's then advances one B per stage instead of one B + W, so the bubble drops
    from (S-1)(F+B+W) to (S-1)(F+B) (ZB-H1; activation memory unchanged).  (Holding W's back further —
    up to S-1-s of them through the steady phase, run in the cool-down — measured no better in
    ``simulate`` for any S, M tried, and holds more (x, dY) pairs.)"""
    warm = min(S - s - 1, M)
    order = [('F', i) for i in range(warm)]
    if kind == '1F1B':
        bw = lambda k: [('BW', k)]  # noqa: E731
    elif kind == 'ZBH1':
        bw = lambda k: [('B', k), ('W', k)]  # noqa: E731
    else:
        raise ValueError(f"unknown pipeline schedule {kind}")
    for k in range(M - warm):
        order += [('F', warm + k)] + bw(k)
    for k in range(M - warm, M):
        order += bw(k)
    return order


def interleaved_units(n, V, P, r):
    """Interleaved 1F1B (virtual pipeline stages) order of rank r of P over n micro-batches and V
    chunks per rank: [('F' | 'B', chunk, micro-batch)] — warm-up 2(P-r-1) + (V-1)P forward units,
    then one forward / one backward unit, then the cool-down; unit k is micro-batch
    (k // PV) P + k % P through chunk (k % PV) // P (reversed for backward).  Needs n % P == 0; else
    the breadth-first order (every micro-batch through chunk 0, then chunk 1, ...)."""
    if V == 1 or n % P != 0:
        return ([('F', v, m) for v in range(V) for m in range(n)] +
                [('B', v, m) for v in reversed(range(V)) for m in range(n)])
    total = n * V
    fch = lambda k: (k % (P * V)) // P  # noqa: E731
    mb = lambda k: (k // (P * V)) * P + k % P  # noqa: E731
    warm = min(total, (P - r - 1) * 2 + (V - 1) * P)
    seq = [('F', k) for k in range(warm)]
    for i in range(total - warm):
        seq += [('F', warm + i), ('B', i)]
    seq += [('B', i) for i in range(total - warm, total)]
    return [(kind, fch(k) if kind == 'F' else V - 1 - fch(k), mb(k)) for kind, k in seq]


def simulate(kind, S, M, f=1.0, b=1.0, w=1.0):
    """Play every stage's schedule_order against the others: returns (makespan, bubble fraction).
    F(s, i) waits for F(s-1, i); B(s, i) for B(s+1, i); W(s, i) for B(s, i); a stage runs its ops
    in order, one at a time; 'BW' costs b + w."""
    cost = {'F': f, 'B': b, 'W': w, 'BW': b + w}
    orders = [schedule_order(kind, S, s, M) for s in range(S)]
    done = {}
    pos = [0] * S
    clock = [0.0] * S
    remaining = sum(len(o) for o in orders)
    while remaining:
        progressed = False
        for s in range(S):
            while pos[s] < len(orders[s]):
                op, i = orders[s][pos[s]]
                if op == 'F':
                    dep = done.get(('F', s - 1, i)) if s > 0 else 0.0
                elif op in ('B', 'BW'):
                    dep = (done.get(('B', s + 1, i)) if s < S - 1 else done.get(('F', s, i)))
                else:
                    dep = done.get(('B', s, i))
                if dep is None:
                    break
                start = max(clock[s], dep)
                clock[s] = start + cost[op]
                done[(op if op != 'BW' else 'B', s, i)] = clock[s]
                if op == 'BW':
                    done[('W', s, i)] = clock[s]
                pos[s] += 1
                remaining -= 1
                progressed = True
        if not progressed:
            raise RuntimeError(f"{kind} schedule deadlocks (S={S}, M={M})")
    makespan = max(clock)
    work = M * (f + b + w)
    return makespan, 1.0 - work / makespan
