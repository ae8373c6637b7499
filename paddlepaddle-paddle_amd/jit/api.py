"""paddle.jit (reference: python/paddle/jit/api.py — to_static:214, not_to_static:357,
save:908, load:1480; translated_layer.py TranslatedLayer).

``to_static(fn)`` (``full_graph=False``, the reference's 3.x default) runs ``fn`` through the SOT
translator — this framework's own opcode translator (jit/opcode_translator.py): the tensor work
between graph breaks becomes static Programs replayed by the Executor under guards, the rest stays
Python (``FLAGS_pa_sot=0`` keeps plain dygraph calls).  ``to_static`` also provides
* a recorded static Program on demand (``concrete_program``) — the same IR ``jit.save``
  serialises (``static/io.py``).  Recording runs the function after ``dy2static`` has rewritten
  its tensor-dependent ``if`` / ``while`` / ``for range`` / ``and``/``or``/``not`` into
  ``cond`` / ``while`` nodes (``jit/dy2static.py``), so the saved program branches per input;
* HIP-graph replay of the forward for inference-shaped calls (``backend='hip_graph'`` or
  ``build_strategy.use_hip_graph``): launch-bound small-batch decoding collapses into one
  graph launch per call;
* ``full_graph=True``: dygraph semantics for calls, the AST-converted recorded Program for
  ``concrete_program`` / ``jit.save``.
``jit.load`` returns a ``TranslatedLayer`` that interprets the saved program without the
Python class that produced it.
"""
import functools

import torch

from ..core.tensor import Tensor, _wrap, _unwrap
from ..nn.layer.layers import Layer
from .dy2static import convert_function, converted_source
from ..static.program import (InputSpec, Program, program_guard, data as _data, _start_recording,
                              _stop_recording, _recorder, default_main_program)

_to_static_enabled = [True]


def enable_to_static(enable_to_static_bool):
    _to_static_enabled[0] = bool(enable_to_static_bool)


def set_code_level(level=100, also_to_stdout=False):
    pass


def set_verbosity(level=0, also_to_stdout=False):
    pass


def ignore_module(modules):
    pass


def not_to_static(func=None):
    def mark(f):
        try:
            f._jst_not_to_static = True
        except (AttributeError, TypeError):
            pass
        return f
    if func is None:
        return mark
    return mark(func)


def _spec_of(x, i):
    if isinstance(x, InputSpec):
        return x
    if isinstance(x, Tensor):
        return InputSpec(x.shape, str(x.dtype).replace('paddle.', ''), name=x.name or f"x{i}")
    return None


class ConcreteProgram:
    def __init__(self, main_program, inputs, outputs, startup_program=None, function=None):
        self.main_program = main_program
        self.startup_program = startup_program or Program()
        self.inputs = inputs
        self.outputs = outputs
        self.function = function
        self.parameters = main_program.all_parameters()


def record_program(fn, input_spec):
    """Records ``fn`` on static Variables built from ``input_spec`` → ConcreteProgram."""
    prog = Program()
    started = _recorder[0] is None
    if started:
        _start_recording()
    try:
        with program_guard(prog):
            feeds = []
            for i, s in enumerate(input_spec):
                name = s.name or f"x{i}"
                shape = [(-1 if (d is None or d < 0) else d) for d in s.shape]
                feeds.append(_data(name, shape, s.dtype))
            out = (convert_function(fn) if _to_static_enabled[0] else fn)(*feeds)
    finally:
        if started:
            _stop_recording()
    outs = out if isinstance(out, (list, tuple)) else [out]
    return ConcreteProgram(prog, feeds, list(outs), function=fn)


class StaticFunction:
    def __init__(self, function, input_spec=None, build_strategy=None, backend=None, full_graph=False, **kw):
        self._fn = function
        self._input_spec = list(input_spec) if input_spec is not None else None
        self._build_strategy = build_strategy
        self._backend = backend
        self._full_graph = full_graph
        self._layer = None
        self._last_specs = None
        self._graphed = None
        self._programs = {}
        functools.update_wrapper(self, function)

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self
        bound = StaticFunction(self._fn.__get__(obj, objtype), self._input_spec, self._build_strategy, self._backend,
                               self._full_graph)
        bound._layer = obj
        return bound

    def _use_graph(self):
        if self._backend == 'hip_graph':
            return True
        bs = self._build_strategy
        return bool(bs is not None and getattr(bs, 'use_hip_graph', False))

    def _use_sot(self):
        from . import sot
        return self._backend == 'sot' or (not self._full_graph and self._backend is None and sot.default_enabled())

    def __call__(self, *args, **kwargs):
        self._last_specs = [_spec_of(a, i) for i, a in enumerate(args)]
        if _to_static_enabled[0] and self._use_sot():
            if getattr(self, '_sot_fn', None) is None:
                from .sot import symbolic_translate
                self._sot_fn = symbolic_translate(self._fn)
            return self._sot_fn(*args, **kwargs)
        if (_to_static_enabled[0] and self._use_graph() and not kwargs and not torch.is_grad_enabled()
                and torch.cuda.is_available()):
            if self._graphed is None:
                from ..device.cuda.graphs import _Graphed
                self._graphed = _Graphed(self._fn)
            return self._graphed(*args)
        return self._fn(*args, **kwargs)

    def get_concrete_program(self, *args, **kwargs):
        specs = [_spec_of(a, i) for i, a in enumerate(args)] if args else (self._input_spec or self._last_specs)
        if specs is None:
            raise ValueError("input_spec is required to build the program")
        key = tuple(specs)
        if key not in self._programs:
            self._programs[key] = record_program(self._fn, specs)
        cp = self._programs[key]
        return cp, cp

    @property
    def concrete_program(self):
        return self.get_concrete_program()[0]

    def concrete_program_specify_input_spec(self, input_spec=None, **kw):
        specs = list(input_spec) if input_spec is not None else (self._input_spec or self._last_specs)
        return self.get_concrete_program(*specs)[0] if specs else None

    @property
    def main_program(self):
        return self.concrete_program.main_program

    @property
    def code(self):
        return converted_source(self._fn)

    @property
    def dygraph_function(self):
        return self._fn

    def rollback(self):
        if self._layer is not None:
            self._layer.forward = self._fn
        return self._fn

    @property
    def inputs(self):
        return self._input_spec


def to_static(function=None, input_spec=None, build_strategy=None, backend=None, full_graph=False, **kwargs):
    def deco(fn):
        if isinstance(fn, Layer):
            sf = StaticFunction(type(fn).forward, input_spec, build_strategy, backend, full_graph)
            fn.forward = sf.__get__(fn, type(fn))
            fn._static_input_spec = input_spec
            return fn
        return StaticFunction(fn, input_spec, build_strategy, backend, full_graph)
    if function is None:
        return deco
    return deco(function)


def save(layer, path, input_spec=None, **configs):
    """Serialise ``layer``'s forward as a program (+ parameters) for ``jit.load`` /
    ``paddle.inference``: ``<path>.pdmodel`` and ``<path>.pdiparams``."""
    from ..static.io import save_inference_model
    if isinstance(layer, Layer):
        fwd = layer.forward
        specs = input_spec
        if specs is None and isinstance(fwd, StaticFunction):
            specs = fwd._input_spec or fwd._last_specs
        if specs is None:
            specs = getattr(layer, '_static_input_spec', None)
        fn = fwd._fn if isinstance(fwd, StaticFunction) else fwd
    elif isinstance(layer, StaticFunction):
        fn, specs = layer._fn, input_spec or layer._input_spec or layer._last_specs
    else:
        fn, specs = layer, input_spec
    if specs is None:
        raise ValueError("jit.save needs input_spec (or a to_static layer that has been called)")
    specs = [s if isinstance(s, InputSpec) else _spec_of(s, i) for i, s in enumerate(specs)]
    cp = record_program(fn, specs)
    outs = cp.outputs
    output_spec = configs.get('output_spec')
    if output_spec is not None:
        keep = {id(_unwrap(o)) for o in output_spec}
        outs = [o for o in outs if id(_unwrap(o)) in keep] or outs
    save_inference_model(path, cp.inputs, outs, program=cp.main_program)


class TranslatedLayer(Layer):
    """A layer rebuilt from ``jit.save`` files; forward interprets the saved program."""

    def __init__(self, program, feed_names, fetch_vars):
        super().__init__()
        self._program = program
        self._feed_names = feed_names
        self._fetch_vars = fetch_vars
        for i, p in enumerate(program.all_parameters()):
            self.add_parameter((p.name or f"param_{i}").replace('.', '_'), p)

    def forward(self, *inputs):
        from ..core.place import current_device
        from ..static.executor import run_program
        from ..static.program import _vid_of
        feed = {n: (x._t if isinstance(x, Tensor) else x) for n, x in zip(self._feed_names, inputs)}
        env = run_program(self._program, feed, current_device(), grad=self.training and torch.is_grad_enabled())
        outs = [_wrap(env[_vid_of(self._program, v)]) for v in self._fetch_vars]
        return outs[0] if len(outs) == 1 else outs

    def program(self, method_name='forward'):
        return self._program


def load(path, **configs):
    from ..static.io import load_inference_model
    prog, feeds, fetches = load_inference_model(path)
    tl = TranslatedLayer(prog, feeds, fetches)
    tl.eval()
    return tl
