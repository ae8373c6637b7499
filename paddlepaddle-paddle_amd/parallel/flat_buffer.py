"""Flat parameter / gradient buffers — the memory layout every MI355X engine here builds on.

A ``FlatBuffer`` re-homes a list of parameters into ONE contiguous device buffer per
dtype (parameters become views at fixed offsets; values and leaf-ness are preserved) and
gives their gradients the same treatment (``p.grad`` is a view into one flat gradient
buffer, so autograd accumulates in place).  Consequences:

* the optimizer update is ONE fused kernel over the whole buffer (``ops.optim.adamw_flat``)
* data-parallel gradient all-reduce / sharding reduce-scatter operate on contiguous
  slices of the flat gradient buffer — no pack/unpack copies, bucket = slice
* sharding stage 1/2/3 partitions are slices of the same buffer (rank r owns
  ``[r*shard, (r+1)*shard)``), padded so every shard is 16-byte aligned and equal sized.

Reference analogue: paddle/fluid/pybind (coalesce_tensor op / FusedAllReduce),
python/paddle/distributed/fleet/meta_parallel/sharding/group_sharded_storage.py.
"""
import torch

ALIGN = 64  # elements; keeps every param view 128-byte aligned for bf16


def _align(n, a=ALIGN):
    return (n + a - 1) // a * a


class FlatBuffer:
    def __init__(self, params, dtype=None, device=None, pad_to_multiple=1, grad_dtype=None):
        """params: list of paddle Parameters (all the same dtype unless ``dtype`` is given)."""
        self.params = list(params)
        assert self.params, "FlatBuffer needs at least one parameter"
        t0 = self.params[0]._t
        self.dtype = dtype or t0.dtype
        self.grad_dtype = grad_dtype or self.dtype
        self.device = device or t0.device
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _align(p._t.numel())
        total = _align(off, ALIGN * pad_to_multiple)
        self.numel = total
        self.data = torch.zeros(total, dtype=self.dtype, device=self.device)
        self.grad = torch.zeros(total, dtype=self.grad_dtype, device=self.device)
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                n = p._t.numel()
                if p._t.grad is not None:  # built lazily after a backward: keep that gradient
                    self.grad[o:o + n].copy_(p._t.grad.reshape(-1))
                view = self.data[o:o + n].view(p._t.shape)
                view.copy_(p._t.detach())
                req = p._t.requires_grad
                p._t.data = view
                if req:
                    p._t.requires_grad_(True)
                p.__dict__['_flat'] = (self, o)
        self.attach_grads()

    def alias_into(self, data_view, grad_view):
        """Move this buffer's storage into caller-provided views (e.g. slices of one larger
        arena) and re-point every parameter / gradient at them."""
        assert data_view.numel() == self.numel and grad_view.numel() == self.numel
        with torch.no_grad():
            data_view.copy_(self.data)
            grad_view.copy_(self.grad)
            self.data, self.grad = data_view, grad_view
            for p, o in zip(self.params, self.offsets):
                req = p._t.requires_grad
                p._t.data = self.data[o:o + p._t.numel()].view(p._t.shape)
                if req:
                    p._t.requires_grad_(True)
        self.attach_grads()

    def attach_grads(self):
        for p, o in zip(self.params, self.offsets):
            if p._t.requires_grad:
                n = p._t.numel()
                p._t.grad = self.grad[o:o + n].view(p._t.shape)

    def grads_attached(self):
        for p, o in zip(self.params, self.offsets):
            g = p._t.grad
            if p._t.requires_grad and (g is None or g.data_ptr() != self.grad[o:o + 1].data_ptr()):
                return False
        return True

    def sync_grads(self):
        """Re-home any gradient autograd allocated outside the flat buffer (e.g. after
        clear_grad(set_to_zero=False)); returns True when a copy was needed."""
        copied = False
        for p, o in zip(self.params, self.offsets):
            g = p._t.grad
            n = p._t.numel()
            slot = self.grad[o:o + n]
            if g is None:
                if p._t.requires_grad:
                    slot.zero_()
                    p._t.grad = slot.view(p._t.shape)
                continue
            if g.data_ptr() != slot.data_ptr():
                slot.copy_(g.reshape(-1))
                p._t.grad = slot.view(p._t.shape)
                copied = True
        return copied

    def data_intact(self):
        return all(p._t.data_ptr() == self.data[o:o + 1].data_ptr() for p, o in zip(self.params, self.offsets))

    def zero_grad(self):
        self.grad.zero_()


def register_grad_ready(p, fn):
    """Call ``fn()`` whenever p's gradient for this backward is complete.

    Fires from torch's post-accumulate-grad hook (ordinary autograd accumulation) AND from
    kernels that accumulate straight into the flat gradient slot (ops.linear's fused
    weight-gradient GEMM, which bypasses AccumulateGrad).  Returns a removable handle."""
    lst = p.__dict__.setdefault('_grad_ready', [])
    lst.append(fn)
    # a gradient whose kernel was deferred (ops.linear grouped weight gradients) is not complete
    # when autograd accumulates its (undefined) value: complete_deferred() fires the hooks later
    h = p._t.register_post_accumulate_grad_hook(lambda t: None if p.__dict__.get('_grad_deferred') else fn())

    class _Handle:
        def remove(self):
            h.remove()
            if fn in lst:
                lst.remove(fn)
    return _Handle()


def _hooks_fire_on_undefined_grad():
    """Does torch run post-accumulate-grad hooks when a Function returns None for a leaf?
    (Observed true on torch 2.x: AccumulateGrad still executes its post hooks.)  Probed once."""
    fired = []

    class _F(torch.autograd.Function):
        @staticmethod
        def forward(ctx, a, w):
            return a * 2

        @staticmethod
        def backward(ctx, g):
            return g * 2, None

    a = torch.ones(2, requires_grad=True)
    w = torch.ones(2, requires_grad=True)
    w.register_post_accumulate_grad_hook(lambda t: fired.append(1))
    _F.apply(a, w).sum().backward()
    return bool(fired)


_HOOKS_FIRE = _hooks_fire_on_undefined_grad()


def notify_grad_ready(p):
    """Called by kernels that wrote p's gradient directly into its flat slot.  When torch itself
    fires the post-accumulate hook for the (undefined) autograd gradient, that hook is the single
    notification; otherwise notify here."""
    if _HOOKS_FIRE:
        return
    for fn in p.__dict__.get('_grad_ready', ()):
        fn()


def defer_grad(p):
    """Mark p's flat-slot gradient as still being computed (its kernel is deferred past the
    autograd node): grad-ready hooks are held until complete_deferred(p)."""
    p.__dict__['_grad_deferred'] = True


def complete_deferred(p):
    """The deferred gradient of p has been written: fire its grad-ready hooks now."""
    if p.__dict__.pop('_grad_deferred', None):
        for fn in list(p.__dict__.get('_grad_ready', ())):
            fn()


# Called by the training engines at the start of their end-of-backward callbacks (and by a
# callback of their own when no engine runs), before any bucket / unit is treated as final:
# producers of deferred gradients flush them here.
_PRE_FINISH = []


def register_pre_finish(fn):
    if fn not in _PRE_FINISH:
        _PRE_FINISH.append(fn)


def run_pre_finish():
    for fn in list(_PRE_FINISH):
        fn()


def flat_grad_slot(p):
    """The flat-buffer gradient view of p if p lives in a FlatBuffer (else None)."""
    if '_flat' not in p.__dict__:
        return None
    g = p._t.grad
    fb, o = p.__dict__['_flat']
    if g is None or fb.grad.untyped_storage().nbytes() == 0 or \
            g.data_ptr() != fb.grad.data_ptr() + o * fb.grad.element_size():
        return None
    return g
