"""Profiler (reference: python/paddle/profiler/profiler.py — Profiler:346, make_scheduler:117,
export_chrome_tracing:215, export_protobuf:268; profiler_statistic.py summary tables).

Two sources, merged into one result:
* host ranges (``RecordEvent``, ProfileStep, Optimization, DataLoader) from the native
  tracer in ``csrc/runtime/tracer.cpp`` (steady-clock ns, per-thread buffers);
* device activity (HIP kernels, memcpy/memset) from the ROCm activity tracer behind
  ``torch.profiler`` (roctracer/rocprofiler-sdk), enabled only for the GPU target.
Results export as Chrome trace JSON and summarise into overview / operator / kernel tables.
"""
import json
import os
import socket
import time
from enum import Enum
from warnings import warn

from .utils import RecordEvent, TracerEventType, _state, _rt, wrap_optimizers
from .timer import benchmark


class SummaryView(Enum):
    DeviceView = 0
    OverView = 1
    ModelView = 2
    DistributedView = 3
    KernelView = 4
    OperatorView = 5
    MemoryView = 6
    MemoryManipulationView = 7
    UDFView = 8


class ProfilerState(Enum):
    CLOSED = 0
    READY = 1
    RECORD = 2
    RECORD_AND_RETURN = 3


class ProfilerTarget(Enum):
    CPU = 0
    GPU = 1
    XPU = 2
    CUSTOM_DEVICE = 3


class SortedKeys(Enum):
    CPUTotal = 0
    CPUAvg = 1
    CPUMax = 2
    CPUMin = 3
    GPUTotal = 4
    GPUAvg = 5
    GPUMax = 6
    GPUMin = 7


def make_scheduler(*, closed, ready, record, repeat=0, skip_first=0):
    def sched(step):
        if step < skip_first:
            return ProfilerState.CLOSED
        step -= skip_first
        period = closed + ready + record
        if period <= 0:
            return ProfilerState.CLOSED
        if repeat > 0 and step // period >= repeat:
            return ProfilerState.CLOSED
        m = step % period
        if m < closed:
            return ProfilerState.CLOSED
        if m < closed + ready:
            return ProfilerState.READY
        return ProfilerState.RECORD_AND_RETURN if m == period - 1 else ProfilerState.RECORD
    return sched


def _default_state_scheduler(step):
    return ProfilerState.RECORD


def _worker_name():
    return f"host_{socket.gethostname()}pid_{os.getpid()}"


def export_chrome_tracing(dir_name, worker_name=None):
    def handle(prof):
        os.makedirs(dir_name, exist_ok=True)
        name = worker_name or _worker_name()
        path = os.path.join(dir_name, f"{name}_time_{time.strftime('%Y_%m_%d_%H_%M_%S')}.paddle_trace.json")
        prof.export(path, 'json')
    return handle


def export_protobuf(dir_name, worker_name=None):
    # no protobuf schema here: the same content is written as JSON with a .pb.json suffix
    def handle(prof):
        os.makedirs(dir_name, exist_ok=True)
        name = worker_name or _worker_name()
        prof.export(os.path.join(dir_name, f"{name}_time_{time.strftime('%Y_%m_%d_%H_%M_%S')}.paddle_trace.pb.json"),
                    'json')
    return handle


def _get_supported_targets():
    import torch
    t = [ProfilerTarget.CPU]
    if torch.cuda.is_available():
        t.append(ProfilerTarget.GPU)
    return t


class ProfilerResult:
    """Merged host + device events; ``events`` are dicts with name/type/start/end (ns)/tid/device."""

    def __init__(self, host, device, steps):
        self.host = host
        self.device = device
        self.steps = steps

    @property
    def events(self):
        return self.host + self.device

    def save(self, path, format='json'):
        trace = []
        pid = os.getpid()
        for e in self.host:
            trace.append({'name': e['name'], 'cat': e['type'], 'ph': 'X', 'pid': pid, 'tid': e['tid'],
                          'ts': e['start'] / 1e3, 'dur': (e['end'] - e['start']) / 1e3})
        for e in self.device:
            trace.append({'name': e['name'], 'cat': e['type'], 'ph': 'X', 'pid': f"GPU {e.get('device', 0)}",
                          'tid': e.get('stream', 0), 'ts': e['start'] / 1e3, 'dur': (e['end'] - e['start']) / 1e3})
        with open(path, 'w') as f:
            json.dump({'traceEvents': trace, 'displayTimeUnit': 'ms',
                       'schemaVersion': 1, 'producer': 'paddle_amd'}, f)
        return path


def _collect_host():
    import ctypes
    lib = _rt()
    n = lib.pa_rt_trace_count()
    if n == 0:
        return []
    buf = (ctypes.c_int64 * (5 * n))()
    got = lib.pa_rt_trace_collect(buf, n)
    names = {}
    out = []
    for i in range(got):
        s, e, nid, typ, tid = buf[5 * i:5 * i + 5]
        if nid not in names:
            names[nid] = lib.pa_rt_trace_name(nid).decode()
        out.append({'name': names[nid], 'type': TracerEventType(typ).name, 'start': s, 'end': e, 'tid': tid})
    return out


class Profiler:
    def __init__(self, *, targets=None, scheduler=None, on_trace_ready=None, record_shapes=False,
                 profile_memory=False, timer_only=False, emit_nvtx=False, custom_device_types=None,
                 with_flops=False):
        supported = _get_supported_targets()
        if targets:
            self.targets = set(t for t in targets if t in supported)
            for t in targets:
                if t not in supported:
                    warn(f"Profiling {t} is not supported in current context.")
        else:
            self.targets = set(supported)
        wrap_optimizers()
        if callable(scheduler):
            self.scheduler = scheduler
        elif isinstance(scheduler, (tuple, list)):
            lo, hi = scheduler
            lo = max(lo, 0)
            if lo >= 1:
                self.scheduler = make_scheduler(closed=max(lo - 1, 0), ready=1, record=hi - lo, repeat=1)
            else:
                self.scheduler = make_scheduler(closed=0, ready=0, record=hi - lo, repeat=1)
        else:
            self.scheduler = _default_state_scheduler
        self.on_trace_ready = on_trace_ready if on_trace_ready is not None else export_chrome_tracing('./profiler_log/')
        self.step_num = 0
        self.previous_state = ProfilerState.CLOSED
        self.current_state = self.scheduler(self.step_num)
        self.record_shapes = record_shapes
        self.profile_memory = profile_memory
        self.timer_only = timer_only
        self.with_flops = with_flops
        self.profiler_result = None
        self._torch_prof = None
        self._step_event = None
        self._t0 = None
        self._steps = []

    # ---- lifecycle
    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *exc):
        self.stop()

    def start(self):
        benchmark().begin()
        if self.timer_only:
            return
        if self.current_state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._begin_record()
        self._open_step()

    def stop(self):
        benchmark().end()
        if self.timer_only:
            return
        self._close_step()
        if self.current_state in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._end_record(handle=True)
        self.current_state = ProfilerState.CLOSED

    def step(self, num_samples=None):
        benchmark().step(num_samples)
        if self.timer_only:
            return
        self._close_step()
        self.previous_state = self.current_state
        self.step_num += 1
        self.current_state = self.scheduler(self.step_num)
        self._transition()
        self._open_step()

    def step_info(self, unit=None):
        return benchmark().step_info(unit)

    # ---- state machine
    def _transition(self):
        prev, cur = self.previous_state, self.current_state
        recording = (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN)
        if prev == ProfilerState.RECORD_AND_RETURN:
            self._end_record(handle=True)
            if cur in recording:
                self._begin_record()
        elif prev in recording and cur not in recording:
            self._end_record(handle=True)
        elif prev not in recording and cur in recording:
            self._begin_record()

    def _begin_record(self):
        lib = _rt()
        lib.pa_rt_trace_clear()
        lib.pa_rt_trace_enable(1)
        _state['recording'] = True
        self._steps = []
        if ProfilerTarget.GPU in self.targets:
            import torch
            acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
            self._torch_prof = torch.profiler.profile(activities=acts, record_shapes=self.record_shapes,
                                                      profile_memory=self.profile_memory,
                                                      with_flops=self.with_flops)
            self._torch_prof.__enter__()
            _state['device_mirror'] = True

    def _end_record(self, handle):
        if not _state['recording']:
            return
        import torch
        device = []
        if self._torch_prof is not None:
            torch.cuda.synchronize()
            self._torch_prof.__exit__(None, None, None)
            _state['device_mirror'] = False
            device = self._device_events(self._torch_prof)
            self._torch_prof_done = self._torch_prof
            self._torch_prof = None
        _rt().pa_rt_trace_enable(0)
        _state['recording'] = False
        self.profiler_result = ProfilerResult(_collect_host(), device, list(self._steps))
        if handle and self.on_trace_ready is not None:
            self.on_trace_ready(self)

    @staticmethod
    def _device_events(tp):
        out = []
        try:
            evs = tp.events()
        except Exception:  # noqa: BLE001
            return out
        for e in evs:
            dt = str(getattr(e, 'device_type', ''))
            if 'CUDA' not in dt and 'HIP' not in dt:
                continue
            start = int(e.time_range.start * 1e3)
            end = int(e.time_range.end * 1e3)
            name = e.name
            kind = 'Memcpy' if 'Memcpy' in name or 'copyBuffer' in name else (
                'Memset' if 'Memset' in name or 'fill' in name.lower() else 'Kernel')
            out.append({'name': name, 'type': kind, 'start': start, 'end': end, 'device': e.device_index,
                        'stream': getattr(e, 'id', 0) % 64})
        return out

    def _open_step(self):
        if _state['recording']:
            self._step_event = RecordEvent(f"ProfileStep#{self.step_num}", TracerEventType.ProfileStep)
            self._step_event.begin()
            self._t0 = time.perf_counter_ns()

    def _close_step(self):
        if self._step_event is not None:
            self._step_event.end()
            if self._t0 is not None:
                self._steps.append((self.step_num, time.perf_counter_ns() - self._t0))
            self._step_event = None

    # ---- outputs
    def export(self, path="", format="json"):
        if self.profiler_result is not None:
            self.profiler_result.save(path, format)

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False, time_unit='ms',
                views=None):
        from .statistic import build_summary
        if self.profiler_result is None:
            return ''
        text = build_summary(self.profiler_result, sorted_by, time_unit, views)
        print(text)
        return text

    def get_profiler_result(self):
        return self.profiler_result
