"""Training-step policy of a recorded ``minimize`` node: gradient merge, data-parallel gradient
reduction and the AMP update, composed in the order the reference program passes apply them.

The reference rewrites the ProgramDesc for these (``c_allreduce_sum`` ops after the backward for
collective data parallelism — fleet/meta_optimizers/raw_program_optimizer.py; gradient-merge
accumulators and a conditional optimizer block — distributed/passes/auto_parallel_gradient_merge.py;
``check_finite_and_unscale`` / ``update_loss_scaling`` — static/amp/decorator.py).  Here a
program is a recorded op list whose ``minimize`` node is executed by ``StaticMinimize``:

  backward of loss (* loss scale) (/ k_steps when averaging)      every run (gradients accumulate)
  on every k-th run:
    all-reduce of the gradients over the data-parallel group (bucketed flat buffers of at most
    ``fuse_grad_size_in_MB``, averaged)
    AMP: unscale + finite check (the found-inf flag max-reduced over the group) + scale update
    optimizer step (gradient clipping inside it), clear_grad
"""
import torch
import torch.distributed as dist


class StaticMinimize:
    def __init__(self, optimizer):
        self._opt = optimizer  # Optimizer, or static.amp.OptimizerWithMixedPrecision
        self.k_steps = 1
        self.avg = True
        self.dp_group = None  # paddle.distributed Group (or None: no reduction)
        self.fuse_grad_size_in_MB = 32
        self._micro = 0
        self.pipeline = None  # static/pipeline.PipelineConfig when the program runs pipelined

    def __getattr__(self, name):
        return getattr(self.__dict__['_opt'], name)

    @property
    def inner_optimizer(self):
        return self._opt

    def _amp(self):
        from .amp import OptimizerWithMixedPrecision
        return self._opt if isinstance(self._opt, OptimizerWithMixedPrecision) else None

    def _plain(self):
        amp = self._amp()
        return amp._optimizer if amp is not None else self._opt

    def _params(self):
        amp = self._amp()
        if amp is not None and amp._params:
            return list(amp._params)
        return list(self._plain()._parameter_list or [])

    def _nranks(self):
        g = self.dp_group
        if g is None or not dist.is_initialized():
            return 1
        return int(getattr(g, 'nranks', None) or dist.get_world_size(getattr(g, 'pg', None)))

    # ---- executed for the recorded minimize node
    def _static_minimize_exec(self, loss):
        div = float(self.k_steps) if (self.k_steps > 1 and self.avg) else 1.0
        amp = self._amp()
        if amp is not None:
            amp._scaled_backward(loss, div)
        elif div != 1.0:
            (loss / div).backward()
        else:
            loss.backward()
        self._micro += 1
        if self._micro % self.k_steps:
            return
        if self._nranks() > 1:
            self._allreduce_grads()
        if amp is not None:
            amp._apply_update(self._sync_found_inf if self._nranks() > 1 else None)
        else:
            opt = self._plain()
            opt.step()
            from .amp import release_grads
            release_grads(opt)

    def _allreduce_grads(self):
        """Average the gradients over the data-parallel group in flat buckets (missing gradients
        are zeros on this rank so every rank issues the same collectives)."""
        pg = getattr(self.dp_group, 'pg', None)
        n = self._nranks()
        ts = []
        for p in self._params():
            t = p._t
            if not t.requires_grad:
                continue
            if t.grad is None:
                t.grad = torch.zeros_like(t)
            ts.append(t.grad)
        cap = max(1, int(self.fuse_grad_size_in_MB * (1 << 20)))
        bucket, size, dt = [], 0, None

        def flush(b):
            if not b:
                return
            flat = torch._utils._flatten_dense_tensors(b)
            dist.all_reduce(flat, group=pg)
            flat.div_(n)
            for g, r in zip(b, torch._utils._unflatten_dense_tensors(flat, b)):
                g.copy_(r)
        for g in ts:
            nb = g.numel() * g.element_size()
            if bucket and (g.dtype != dt or size + nb > cap):
                flush(bucket)
                bucket, size = [], 0
            bucket.append(g)
            size += nb
            dt = g.dtype
        flush(bucket)

    def _sync_found_inf(self, found):
        pg = getattr(self.dp_group, 'pg', None)
        p = self._params()
        dev = p[0]._t.device if p else torch.device('cpu')
        t = torch.tensor([1.0 if found else 0.0], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
        return bool(t.item() > 0)


def minimize_node(program):
    """The (last) recorded minimize node of a program, or None."""
    for n in reversed(program.nodes):
        if n.kind == 'minimize':
            return n
    return None


def step_policy(program):
    """The StaticMinimize executing the program's minimize node (installed on first use)."""
    n = minimize_node(program)
    if n is None:
        raise ValueError("the program has no optimizer.minimize(...) node")
    if not isinstance(n.target, StaticMinimize):
        n.target = StaticMinimize(n.target)
    return n.target
