"""RecordEvent & helpers (reference: python/paddle/profiler/utils.py — RecordEvent:40,
load_profiler_result, in_profiler_mode, wrap_optimizers).

Host ranges go to the native tracer (``csrc/runtime/tracer.cpp``: per-thread buffers, no
lock on the hot path); while a Profiler is recording, ranges are also mirrored into the
device profiler's timeline (``torch.profiler.record_function``) so host ranges and HIP kernels
line up in one trace.
"""
import functools
import json
from contextlib import ContextDecorator
from enum import Enum


class TracerEventType(Enum):
    Operator = 0
    Dataloader = 1
    ProfileStep = 2
    CudaRuntime = 3
    Kernel = 4
    Memcpy = 5
    Memset = 6
    UserDefined = 7
    OperatorInner = 8
    Forward = 9
    Backward = 10
    Optimization = 11
    Communication = 12
    PythonOp = 13
    PythonUserDefined = 14


_state = {'recording': False, 'device_mirror': False}


def in_profiler_mode():
    return _state['recording']


def _rt():
    from .. import _runtime
    return _runtime.lib()


class RecordEvent(ContextDecorator):
    def __init__(self, name, event_type=TracerEventType.PythonUserDefined):
        self.name = name
        self.event_type = event_type
        self._id = None
        self._dev = None

    def begin(self):
        if not _state['recording']:
            return
        lib = _rt()
        if self._id is None:
            self._id = lib.pa_rt_trace_intern(self.name.encode())
        lib.pa_rt_trace_push(self._id, self.event_type.value)
        if _state['device_mirror']:
            import torch
            self._dev = torch.profiler.record_function(self.name)
            self._dev.__enter__()

    def end(self):
        if self._dev is not None:
            self._dev.__exit__(None, None, None)
            self._dev = None
        if _state['recording'] and self._id is not None:
            _rt().pa_rt_trace_pop()

    def __enter__(self):
        self.begin()
        return self

    def __exit__(self, *exc):
        self.end()
        return False


def load_profiler_result(filename):
    """Loads a trace written by ``export_chrome_tracing`` / ``Profiler.export`` (JSON)."""
    with open(filename) as f:
        return json.load(f)


_wrapped = [False]


def wrap_optimizers():
    """Times every ``Optimizer.step`` as an Optimization event."""
    if _wrapped[0]:
        return
    from ..optimizer.optimizer import Optimizer
    orig = Optimizer.step

    @functools.wraps(orig)
    def step(self, *a, **k):
        with RecordEvent(f"{type(self).__name__}.step", TracerEventType.Optimization):
            return orig(self, *a, **k)
    Optimizer.step = step
    _wrapped[0] = True
