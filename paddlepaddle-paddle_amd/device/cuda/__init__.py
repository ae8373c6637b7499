"""paddle.device.cuda (reference: python/paddle/device/cuda/__init__.py): device queries,
allocator statistics (torch's caching allocator, or the native auto-growth allocator of
allocator.py when enabled), streams, and HIP graphs (graphs.py)."""
import torch

from . import allocator as native_allocator

from .. import Stream, Event, current_stream, synchronize as _sync, stream_guard as _sg, _dev  # noqa: F401
from .graphs import CUDAGraph, is_cuda_graph_supported, wrap_cuda_graph, capture_train_step, TrainStepGraph  # noqa: F401


def synchronize(device=None):
    _sync(device)


def device_count():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def empty_cache():
    from ...ops.workspace import release_all
    release_all()  # kernel scratch (dS^T, split-K partials) no captured graph still addresses
    if native_allocator.is_enabled():
        native_allocator.empty_cache(torch.cuda.current_device())
    elif torch.cuda.is_available():
        torch.cuda.empty_cache()


def _idx(device):
    return _dev(device)


def max_memory_allocated(device=None):
    if native_allocator.is_enabled():
        return native_allocator.stats(_idx(device))['peak_allocated']
    return torch.cuda.max_memory_allocated(_idx(device))


def max_memory_reserved(device=None):
    if native_allocator.is_enabled():
        return native_allocator.stats(_idx(device))['peak_reserved']
    return torch.cuda.max_memory_reserved(_idx(device))


def memory_allocated(device=None):
    if native_allocator.is_enabled():
        return native_allocator.stats(_idx(device))['allocated']
    return torch.cuda.memory_allocated(_idx(device))


def memory_reserved(device=None):
    if native_allocator.is_enabled():
        return native_allocator.stats(_idx(device))['reserved']
    return torch.cuda.memory_reserved(_idx(device))


def reset_max_memory_allocated(device=None):
    if native_allocator.is_enabled():
        native_allocator.reset_peak(_idx(device))
        return
    torch.cuda.reset_peak_memory_stats(_idx(device))


reset_max_memory_reserved = reset_max_memory_allocated


def memory_summary(device=None):
    return torch.cuda.memory_summary(_idx(device))


def stream_guard(stream):
    return _sg(stream)


class _Props:
    def __init__(self, p):
        self.name = p.name
        self.major, self.minor = p.major, p.minor
        self.total_memory = p.total_memory
        self.multi_processor_count = p.multi_processor_count
        self.gcnArchName = getattr(p, 'gcnArchName', '')

    def __repr__(self):
        return (f"_gpuDeviceProperties(name='{self.name}', arch='{self.gcnArchName}', major={self.major}, "
                f"minor={self.minor}, total_memory={self.total_memory // (1 << 20)}MB, "
                f"multi_processor_count={self.multi_processor_count})")


def get_device_properties(device=None):
    return _Props(torch.cuda.get_device_properties(_idx(device)))


def get_device_name(device=None):
    return torch.cuda.get_device_name(_idx(device))


def get_device_capability(device=None):
    return torch.cuda.get_device_capability(_idx(device))


def get_rng_state(device=None):
    from ...core.tensor import _wrap
    return _wrap(torch.cuda.get_rng_state(_idx(device)))


def set_rng_state(state, device=None):
    from ...core.tensor import _unwrap
    torch.cuda.set_rng_state(_unwrap(state).cpu(), _idx(device))
