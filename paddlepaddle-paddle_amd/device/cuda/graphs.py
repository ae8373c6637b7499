"""HIP graph capture/replay (reference: python/paddle/device/cuda/graphs.py CUDAGraph,
cuda_graphed_layer.py; the role CINN's whole-graph compilation plays for the reference's
static training, here done by replaying a captured hipGraph).

Launch-bound inner loops (small decode steps, optimizer sweeps over many tensors) and whole
TRAINING STEPS (forward + backward + fused optimizer, ``TrainStepGraph``) are captured once into a
hipGraph and replayed with one launch.  Inputs are copied into static buffers; all kernels of the
captured region (including this framework's ctypes-launched HIP kernels, which launch on the
current — i.e. capturing — stream) become graph nodes.
"""
import torch


def is_cuda_graph_supported():
    return torch.cuda.is_available()


class CUDAGraph:
    def __init__(self, place=None, mode="thread_local", pool_id=None):
        self._g = torch.cuda.CUDAGraph()
        self._pool = pool_id
        self._stream = None
        self._ctx = None

    def capture_begin(self):
        self._stream = torch.cuda.Stream()
        self._stream.wait_stream(torch.cuda.current_stream())
        self._ctx = torch.cuda.stream(self._stream)
        self._ctx.__enter__()
        self._g.capture_begin(pool=self._pool)

    def capture_end(self):
        self._g.capture_end()
        self._ctx.__exit__(None, None, None)
        torch.cuda.current_stream().wait_stream(self._stream)

    def replay(self):
        self._g.replay()

    def reset(self):
        self._g.reset()

    def pool(self):
        return self._g.pool()

    def print_to_dot_files(self, dirname, flags=None):
        import os
        os.makedirs(str(dirname), exist_ok=True)
        self._g.debug_dump(os.path.join(str(dirname), 'graph.dot'))


def _flatten(obj, out):
    from ...core.tensor import Tensor
    if isinstance(obj, Tensor):
        out.append(obj._t)
    elif isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _flatten(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _flatten(o, out)
    return out


class _Graphed:
    """Forward-only graphed callable: first ``warmup`` calls run eagerly, the next captures,
    later calls copy inputs into the static buffers and replay."""

    def __init__(self, fn, warmup=2):
        self.fn = fn
        self.warmup = warmup
        self.calls = 0
        self.graph = None
        self.static_in = None
        self.static_out = None
        self.sig = None

    def __call__(self, *args):
        from ...core.tensor import _wrap
        ins = _flatten(args, [])
        sig = tuple((t.shape, t.dtype, t.device) for t in ins)
        if self.graph is not None and sig != self.sig:
            self.graph = None  # shapes changed: recapture
            self.calls = 0
        if self.graph is None:
            self.calls += 1
            if self.calls <= self.warmup or not torch.cuda.is_available():
                return self.fn(*args)
            self.sig = sig
            self.static_in = [t.clone() for t in ins]
            it = iter(self.static_in)

            def rebuild(obj):
                from ...core.tensor import Tensor
                if isinstance(obj, Tensor):
                    return _wrap(next(it))
                if isinstance(obj, torch.Tensor):
                    return next(it)
                if isinstance(obj, (list, tuple)):
                    return type(obj)(rebuild(o) for o in obj)
                if isinstance(obj, dict):
                    return {k: rebuild(v) for k, v in obj.items()}
                return obj
            static_args = rebuild(args)
            g = CUDAGraph()
            torch.cuda.synchronize()
            g.capture_begin()
            try:
                self.static_out = self.fn(*static_args)
            finally:
                g.capture_end()
            self.graph = g
        for dst, src in zip(self.static_in, ins):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out


def wrap_cuda_graph(function, mode="thread_local", memory_pool="default"):
    return _Graphed(function)


class TrainStepGraph:
    """A whole training step (``step_fn()``: forward, loss, backward, optimizer step, clear_grad,
    returning the loss) captured into one hipGraph and replayed per call.

    The first ``warmup`` calls run eagerly on a side stream (allocator pools, flat-buffer set-up,
    library kernel selection and lazily-built optimizer state all happen there, none inside the
    capture); the next call captures; every later call is ``graph.replay()``.  ``step_fn`` must
    read its inputs from fixed tensors (copy the next batch into them before calling) and must not
    synchronise with the host; per-step host values frozen at capture are refused: dropout inside
    the step is graph-safe: the HIP dropout kernels mix a device-resident generation counter into
    their host-drawn seeds (csrc/common.h rng_mix), and the captured graph advances that counter as
    its first node, so every replay draws fresh keep-masks (a step's backward still regenerates its
    forward's).  The fused optimizers read their learning rate from a device scalar that an
    ``on_replay`` hook refills from ``get_lr()`` before each replay (LR schedulers stepped on the
    host between calls take effect), and their host step counters advance after each replay.
    Returns the static loss tensor (its value updates on every replay).
    """

    def __init__(self, step_fn, warmup=3):
        self.step_fn = step_fn
        self.warmup = warmup
        self.calls = 0
        self.graph = None
        self.out = None
        self.hooks = []  # (pre, post) host callbacks registered through on_replay() during capture
        self.replays = 0

    def _pre(self):
        for pre, _ in self.hooks:
            if pre is not None:
                pre()

    def __call__(self):
        global _CAPTURE_HOOKS
        if not torch.cuda.is_available():
            return self.step_fn()
        if self.graph is not None:
            self._pre()
            self.graph.replay()
            self.replays += 1
            for _, post in self.hooks:
                if post is not None:
                    post()
            return self.out
        self.calls += 1
        if self.calls <= self.warmup:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                out = self.step_fn()
            torch.cuda.current_stream().wait_stream(s)
            return out
        gen = install_rng_generation()
        torch.cuda.synchronize()
        g = CUDAGraph()
        hooks, _CAPTURE_HOOKS = [], []
        g.capture_begin()
        try:
            if gen is not None:
                gen.add_(1)  # first node of every replay: a fresh dropout stream per step
                _RNG_CAPTURE.add(torch.cuda.current_device())
            self.out = self.step_fn()
        finally:
            _RNG_CAPTURE.discard(torch.cuda.current_device())
            g.capture_end()
            hooks, _CAPTURE_HOOKS = _CAPTURE_HOOKS, None
        self.hooks = hooks
        self.graph = g
        # the captured step has not executed yet: run it once for this call (its host-side
        # bookkeeping already ran during the capture, so no post hooks for this one)
        self._pre()
        g.replay()
        self.replays = 1
        return self.out


_CAPTURE_HOOKS = None  # list while a TrainStepGraph captures, else None


def on_replay(pre=None, post=None):
    """Register host callbacks with the TrainStepGraph being captured.

    ``pre()`` runs before every replay and refreshes device-resident scalars from host state (the
    optimizers fill their device learning rate from ``get_lr()``, so an LR scheduler stepped on the
    host between replays takes effect); ``post()`` runs after every replay but the first and
    advances host counters whose update the captured step's Python code performed once, at capture
    (optimizer step counts, host copies of the bias-correction powers).  Returns True when a
    capture took the hooks; False (nothing registered) outside a TrainStepGraph capture, where a
    caller keeps its host values (frozen into a raw ``CUDAGraph``)."""
    if _CAPTURE_HOOKS is None:
        return False
    _CAPTURE_HOOKS.append((pre, post))
    return True


def capture_train_step(step_fn, warmup=3):
    """``TrainStepGraph(step_fn, warmup)``: the training step as one replayable hipGraph."""
    return TrainStepGraph(step_fn, warmup)


_RNG_GEN = {}  # device index -> int32 [1] generation counter read by the HIP dropout kernels
# devices whose graph being captured advances that counter as its first node (a TrainStepGraph
# capture): only there is a host-drawn dropout seed safe to freeze into the graph
_RNG_CAPTURE = set()


def install_rng_generation(device=None):
    """The device-resident dropout generation counter (created and handed to the norm / activation
    / flash-attention kernel modules on first use; 0 until a captured step advances it, so eager
    steps keep their host-drawn streams).  None when the HIP kernel library is not loaded."""
    from ...ops import _native as N
    if N._load() is None:
        return None
    dev = torch.device('cuda', torch.cuda.current_device() if device is None else device)
    gen = _RNG_GEN.get(dev.index)
    if gen is None:
        gen = torch.zeros(1, dtype=torch.int32, device=dev)
        for fn in ('pa_norm_set_rng_gen', 'pa_act_set_rng_gen', 'pa_flash_set_rng_gen', 'pa_flash_ds_set_rng_gen'):
            N.check(getattr(N.lib, fn)(N.ptr(gen)), fn)
        _RNG_GEN[dev.index] = gen
    return gen


def rng_generation(device=None):
    """The generation counter tensor of ``device`` (None before the first captured step)."""
    return _RNG_GEN.get(torch.cuda.current_device() if device is None else device)


def host_rng_guard(what):
    """Raise when a kernel would freeze a host-drawn dropout seed into a graph being captured
    without a per-replay advance of the device generation counter (install_rng_generation).  Only a
    TrainStepGraph capture adds that advance; a raw CUDAGraph / wrap_cuda_graph / DecodeStepGraph
    capture raises even after a TrainStepGraph created the counter on this device."""
    if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing() and \
            torch.cuda.current_device() not in _RNG_CAPTURE:
        raise RuntimeError(f"{what}: dropout seeds are drawn on the host and would be frozen into the "
                           "captured graph (every replay would reuse one mask); capture the step without "
                           "dropout or run it eagerly")


class DecodeStepGraph:
    """One generation (decode) step of a cached model captured into a hipGraph and replayed per
    token — the launch-bound small-batch decode loop becomes one graph launch.

    ``step_fn(x, time_step)`` runs the model on the new tokens ``x`` at position ``time_step`` (a
    device int tensor, e.g. ``FusedMultiTransformer(x, caches=..., time_step=...)``) and returns its
    output; KV caches are updated in place by the model.  The graph reads ``x`` from a static
    buffer and ``time_step`` from a device counter it advances by one as its last node, so each
    call is ``copy new tokens -> replay`` with no host-side position bookkeeping.  ``warmup``
    eager steps run first (allocator pools, kernel selection); the first captured call also
    produces that step's output.  Host-side cache features (beam_offset, pre_caches) are refused.
    Any other per-step tensor ``step_fn`` uses (an attention mask, rotary tables, sequence
    lengths) is captured by address: keep it in a static buffer and refill it in place before the
    call — a new tensor created per step is not seen by the replay.
    """

    def __init__(self, step_fn, x_example, start_step, warmup=1):
        self.step_fn = step_fn
        self.x = x_example.clone()
        self.time_step = torch.tensor([int(start_step)], dtype=torch.int32, device=self.x.device)
        self.warmup = warmup
        self.graph = None
        self.out = None

    def __call__(self, x_new):
        from ...core.tensor import Tensor, _wrap
        xt = x_new._t if isinstance(x_new, Tensor) else x_new
        self.x.copy_(xt)
        if self.graph is not None:
            self.graph.replay()
            return self.out
        if self.warmup > 0:
            self.warmup -= 1
            out = self.step_fn(_wrap(self.x), _wrap(self.time_step))
            self.time_step.add_(1)
            return out
        torch.cuda.synchronize()
        g = CUDAGraph()  # captures on its own side stream
        g.capture_begin()
        try:
            self.out = self.step_fn(_wrap(self.x), _wrap(self.time_step))
            self.time_step.add_(1)
        finally:
            g.capture_end()
        self.graph = g
        g.replay()
        return self.out
