"""Bytecode-level dygraph-to-static translation ("SOT", reference python/paddle/jit/sot/ —
symbolic_translate, the default ``to_static(full_graph=False)`` mode of Paddle 3.x).

The reference simulates the function's bytecode, builds a static program from the tensor
operations it can follow and falls back to dygraph around what it cannot ("graph breaks"),
guarding each captured program on the inputs it was built for.  Two front ends:

* ``frontend='opcode'`` (default): this framework's own opcode translator
  (jit/opcode_translator.py) — a CPython 3.10 bytecode interpreter that records each region of
  the frame between graph breaks into a static ``Program`` with the static recorder, runs it on
  the Executor and replays it under guards;
* ``frontend='dynamo'``: CPython frame evaluation through ``torch._dynamo`` as the bytecode front
  end, every captured FX graph recorded into a static ``Program`` on meta Variables shaped like
  the graph's inputs (a graph the recorder cannot follow runs as captured).

Either way each call interprets the captured Programs with the Executor's runner
(static/executor.py ``run_program``): recorded GEMMs substituted onto the hand-written MFMA kernels,
the IR fusion passes (attention -> flash kernel, LayerNorm / skip-LayerNorm -> norm kernels, fc +
bias + act -> GEMM epilogue, softmax) applied on GPU programs, autograd kept when gradients are
enabled.  A translation failure never changes results.

Usage: ``paddle.jit.sot.symbolic_translate(fn)(*args)``, ``paddle.jit.to_static(fn, backend='sot')``
(or ``full_graph=False`` with ``FLAGS_pa_sot=1``).
"""
from ..framework.flags import pa_flag  # noqa: E402
import functools
import os

import torch

from ..core.tensor import SOT_ACTIVE

_STATS = {'graphs': 0, 'recorded': 0, 'fallback': 0, 'calls': 0}


def stats():
    """Counters of the translators: captured graphs (regions), graphs recorded into Programs,
    graphs left on the FX fallback, and calls served by recorded Programs."""
    from .opcode_translator import stats as _ot
    o = _ot()
    return {'graphs': _STATS['graphs'] + o['regions'], 'recorded': _STATS['recorded'] + o['recorded'],
            'fallback': _STATS['fallback'], 'calls': _STATS['calls'] + o['runs'], 'breaks': o['breaks'],
            'eager_calls': o['eager_calls']}


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


def symbolic_translate(fn=None, training=True, frontend=None, **kwargs):
    """Translate ``fn`` (a function or a Layer's bound forward) at the bytecode level: tensor work
    runs as captured static Programs on the Executor, the rest of the frame stays Python.
    ``frontend``: 'opcode' (this framework's translator, default) or 'dynamo'."""
    fe = frontend or pa_flag('sot_frontend')

    def wrap(f):
        if fe != 'dynamo':
            from .opcode_translator import OpcodeTranslator
            tr = OpcodeTranslator(f)

            @functools.wraps(f)
            def run_ot(*args, **kw):
                return tr(*args, **kw)
            run_ot._sot_translator = tr
            return run_ot
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
