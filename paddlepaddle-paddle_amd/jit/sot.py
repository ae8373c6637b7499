"""Bytecode-level dygraph-to-static translation ("SOT", reference python/paddle/jit/sot/ —
symbolic_translate, the default ``to_static(full_graph=False)`` mode of Paddle 3.x).

The reference simulates the function's bytecode, builds a static program from the tensor
operations it can follow and falls back to dygraph around what it cannot ("graph breaks"),
guarding each captured program on the inputs it was built for.  Here the bytecode front end is
CPython frame evaluation through ``torch._dynamo`` (the function's bytecode is symbolically
executed; unsupported Python — data-dependent branches on tensor values, prints, calls into
extensions — becomes a graph break and runs eagerly; guards re-translate on new shapes / types),
and the back end is this framework's own static stack:

* every captured FX graph is recorded into a static ``Program`` (static/program.py) on meta
  Variables shaped like the graph's inputs, and
* each call interprets that Program with the Executor's runner (static/executor.py
  ``run_program``): recorded GEMMs substituted onto the hand-written MFMA kernels, the IR fusion
  passes (attention -> flash kernel, LayerNorm / skip-LayerNorm -> norm kernels, fc + bias + act ->
  GEMM epilogue, softmax) applied on GPU programs, autograd kept when gradients are enabled.

While a frame is being translated the paddle ops take their torch composite forms
(``ops.use_hip`` is False under tracing), so the captured graphs are whole torch-op graphs and the
Executor maps them back onto the HIP kernels.  A graph the recorder cannot follow runs as the
captured FX graph (eager torch ops): a translation failure never changes results.

Usage: ``paddle.jit.sot.symbolic_translate(fn)(*args)``, ``paddle.jit.to_static(fn, backend='sot')``
(or ``full_graph=False`` with ``PADDLE_AMD_SOT=1``).
"""
from ..framework.flags import pa_flag  # noqa: E402
import functools
import os

import torch

from ..core.tensor import SOT_ACTIVE

_STATS = {'graphs': 0, 'recorded': 0, 'fallback': 0, 'calls': 0}


def stats():
    """Counters of the translator: captured graphs, graphs recorded into Programs, graphs left on
    the FX fallback, and calls served by recorded Programs."""
    return dict(_STATS)


def _paddle_dtype(dt):
    return {torch.float32: 'float32', torch.float16: 'float16', torch.bfloat16: 'bfloat16', torch.float64: 'float64',
            torch.int64: 'int64', torch.int32: 'int32', torch.bool: 'bool', torch.int8: 'int8',
            torch.uint8: 'uint8'}.get(dt)


class _CapturedGraph:
    """One graph of the translated frame: its FX module, and the static Program it was recorded
    into (built on the first call)."""

    def __init__(self, gm, example_inputs):
        self.gm = gm
        self.prog = None
        self.fallback = False
        self.feed_names = None
        self.out_refs = None
        self.specs = []
        for t in example_inputs:
            if not isinstance(t, torch.Tensor) or any(not isinstance(s, int) for s in t.shape):
                self.fallback = True  # symbolic sizes / non-tensor inputs: keep the FX graph
                break
            self.specs.append((tuple(t.shape), t.dtype))
        _STATS['graphs'] += 1

    def _record(self):
        from ..static.program import Program, program_guard, data, _start_recording, _stop_recording, _recorder
        prog = Program()
        started = _recorder[0] is None
        if started:
            _start_recording()
        try:
            with program_guard(prog):
                feeds, names = [], []
                for i, (shape, dt) in enumerate(self.specs):
                    pdt = _paddle_dtype(dt)
                    if pdt is None:
                        raise TypeError(f"sot: unsupported input dtype {dt}")
                    names.append(f"sot_in{i}")
                    feeds.append(data(names[-1], list(shape), pdt))
                metas = [f._t for f in feeds]
                out = self.gm(*metas)
        finally:
            if started:
                _stop_recording()
        outs = list(out) if isinstance(out, (list, tuple)) else [out]
        refs = []
        by_id = {id(m): i for i, m in enumerate(metas)}
        for o in outs:
            if isinstance(o, torch.Tensor) and o.is_meta:
                if id(o) in by_id:
                    refs.append(('in', by_id[id(o)]))
                else:
                    vid = prog._val.get(id(o))
                    if vid is None:
                        raise RuntimeError("sot: graph output not produced by a recorded op")
                    refs.append(('v', vid))
            else:
                refs.append(('c', o))
        self.prog, self.feed_names, self.out_refs = prog, names, refs
        self.tuple_out = isinstance(out, (list, tuple))

    def __call__(self, *args):
        if not self.fallback and self.prog is None:
            try:
                self._record()
                _STATS['recorded'] += 1
            except Exception:  # noqa: BLE001 — the recorder cannot follow this graph: run it as captured
                self.fallback = True
                _STATS['fallback'] += 1
        if self.fallback:
            return self.gm(*args)
        from ..static.executor import run_program
        dev = args[0].device if args and isinstance(args[0], torch.Tensor) else None
        env = run_program(self.prog, dict(zip(self.feed_names, args)), dev, grad=torch.is_grad_enabled())
        _STATS['calls'] += 1
        res = []
        for kind, v in self.out_refs:
            res.append(args[v] if kind == 'in' else env[v] if kind == 'v' else v)
        return tuple(res) if self.tuple_out else res[0]


def _backend(gm, example_inputs):
    return _CapturedGraph(gm, example_inputs)


def symbolic_translate(fn=None, training=True, **kwargs):
    """Translate ``fn`` (a function or a Layer's bound forward) at the bytecode level: tensor work
    runs as captured static Programs on the Executor, the rest of the frame stays Python."""
    def wrap(f):
        compiled = torch.compile(f, backend=_backend, fullgraph=False, dynamic=False)

        @functools.wraps(f)
        def run(*args, **kw):
            prev, SOT_ACTIVE[0] = SOT_ACTIVE[0], True
            try:
                return compiled(*args, **kw)
            finally:
                SOT_ACTIVE[0] = prev
        run._sot_compiled = compiled
        return run
    if fn is None:
        return wrap
    return wrap(fn)


def default_enabled():
    return pa_flag('sot')


def reset():
    """Drop every translation (guards and captured graphs)."""
    torch._dynamo.reset()


__all__ = ['symbolic_translate', 'stats', 'reset']
