"""paddle.device (reference: python/paddle/device/__init__.py — set_device:265, get_device:297,
Event:445, Stream:617, current_stream:833, set_stream:884, stream_guard:929, synchronize:989).

Streams and events are HIP streams/events of the MI355X (one process per GPU); a Stream wraps
the runtime's stream object so paddle code, our ctypes kernels (which launch on the *current*
stream) and RCCL collectives all order against the same queue.
"""
import torch

from ..core.place import (set_device, get_device, CPUPlace, CUDAPlace, CUDAPinnedPlace, XPUPlace,  # noqa: F401
                          IPUPlace, CustomPlace, is_compiled_with_cuda, is_compiled_with_rocm,
                          is_compiled_with_xpu, is_compiled_with_custom_device, is_compiled_with_cinn,
                          is_compiled_with_distribute, to_device, current_device)


def is_compiled_with_ipu():
    return False


def get_cudnn_version():
    return None  # MIOpen, not cuDNN


def get_all_device_type():
    return ['cpu', 'gpu'] if torch.cuda.is_available() else ['cpu']


def get_all_custom_device_type():
    return []


def get_available_device():
    if not torch.cuda.is_available():
        return []
    return [f'gpu:{i}' for i in range(torch.cuda.device_count())]


def get_available_custom_device():
    return []


def get_device_count():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def _dev(device):
    if device is None:
        return current_device()
    return to_device(device)


class Event:
    """HIP event (timing optional)."""

    def __init__(self, device=None, enable_timing=False, blocking=False, interprocess=False):
        self.device = _dev(device)
        self.event_base = torch.cuda.Event(enable_timing=enable_timing, blocking=blocking, interprocess=interprocess)

    def record(self, stream=None):
        s = stream.stream_base if isinstance(stream, Stream) else stream
        self.event_base.record(s if s is not None else torch.cuda.current_stream(self.device))

    def query(self):
        return self.event_base.query()

    def elapsed_time(self, end_event):
        return self.event_base.elapsed_time(end_event.event_base)

    def synchronize(self):
        self.event_base.synchronize()

    def __repr__(self):
        return f"<paddle.device.Event on {self.device}>"


class Stream:
    """HIP stream.  ``priority``: paddle uses 1 (high) / 2 (normal); mapped to HIP priorities."""

    def __init__(self, device=None, priority=2, stream_base=None):
        if stream_base is not None:
            self.stream_base = stream_base
            self.device = stream_base.device
            return
        self.device = _dev(device)
        self.stream_base = torch.cuda.Stream(device=self.device, priority=-1 if priority == 1 else 0)

    def wait_event(self, event):
        self.stream_base.wait_event(event.event_base)

    def wait_stream(self, stream):
        self.stream_base.wait_stream(stream.stream_base)

    def record_event(self, event=None):
        if event is None:
            event = Event(self.device)
        event.record(self)
        return event

    def query(self):
        return self.stream_base.query()

    def synchronize(self):
        self.stream_base.synchronize()

    @property
    def cuda_stream(self):
        return self.stream_base.cuda_stream

    def __eq__(self, other):
        return isinstance(other, Stream) and self.stream_base == other.stream_base

    def __hash__(self):
        return hash(self.stream_base)

    def __repr__(self):
        return f"<paddle.device.Stream {self.stream_base.cuda_stream:#x} on {self.device}>"


def current_stream(device=None):
    return Stream(stream_base=torch.cuda.current_stream(_dev(device)))


def set_stream(stream):
    prev = current_stream(stream.device)
    torch.cuda.set_stream(stream.stream_base)
    return prev


class stream_guard:
    def __init__(self, stream=None):
        self.stream = stream
        self._ctx = None

    def __enter__(self):
        if self.stream is not None:
            self._ctx = torch.cuda.stream(self.stream.stream_base)
            self._ctx.__enter__()
        return self.stream

    def __exit__(self, *a):
        if self._ctx is not None:
            self._ctx.__exit__(*a)


def synchronize(device=None):
    if torch.cuda.is_available():
        torch.cuda.synchronize(_dev(device) if device is not None else None)


from . import cuda  # noqa: F401,E402
