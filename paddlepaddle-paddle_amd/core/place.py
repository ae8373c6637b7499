"""Places and the current device.

Reference: python/paddle/device/__init__.py (set_device/get_device), paddle/phi/common/place.h.
On this framework a "gpu" place is a HIP device of the MI355X node; one process drives
one GPU (LOCAL_RANK), so the default place is ``gpu:LOCAL_RANK`` when a GPU is visible.
"""
import os

import torch


class Place:
    __slots__ = ('_dev',)

    def __init__(self, dev):
        self._dev = torch.device(dev)

    def is_cpu_place(self):
        return self._dev.type == 'cpu'

    def is_gpu_place(self):
        return self._dev.type == 'cuda'

    def is_cuda_pinned_place(self):
        return False

    def is_custom_place(self):
        return False

    def is_xpu_place(self):
        return False

    def gpu_device_id(self):
        return self._dev.index or 0

    def get_device_id(self):
        return self._dev.index or 0

    def __eq__(self, other):
        return isinstance(other, Place) and other._dev == self._dev

    def __hash__(self):
        return hash(self._dev)

    def __repr__(self):
        if self._dev.type == 'cpu':
            return 'Place(cpu)'
        return f'Place(gpu:{self._dev.index or 0})'

    __str__ = __repr__


class CPUPlace(Place):
    __slots__ = ()

    def __init__(self):
        super().__init__('cpu')


class CUDAPlace(Place):
    __slots__ = ()

    def __init__(self, idx=0):
        super().__init__(f'cuda:{idx}')


class CUDAPinnedPlace(Place):
    __slots__ = ()

    def __init__(self):
        super().__init__('cpu')

    def is_cuda_pinned_place(self):
        return True

    def __repr__(self):
        return 'Place(gpu_pinned)'


XPUPlace = CUDAPlace
CustomPlace = CUDAPlace
IPUPlace = CPUPlace


def _initial_device():
    if torch.cuda.is_available():
        idx = int(os.environ.get('LOCAL_RANK', os.environ.get('FLAGS_selected_gpus', '0').split(',')[0] or 0))
        idx = idx % max(torch.cuda.device_count(), 1)
        return torch.device('cuda', idx)
    return torch.device('cpu')


_current = None


def current_device():
    """The torch.device new tensors are created on (paddle's expected place)."""
    global _current
    if _current is None:
        _current = _initial_device()
        if _current.type == 'cuda':
            torch.cuda.set_device(_current)
            from ..ops.gemm_tuning import apply_tuned_db
            apply_tuned_db()
    return _current


def to_device(place):
    """Normalise a paddle place spec (Place, 'gpu:0', 'cpu', int) to torch.device."""
    if place is None:
        return current_device()
    if isinstance(place, Place):
        return place._dev
    if isinstance(place, torch.device):
        return place
    if isinstance(place, int):
        return torch.device('cuda', place)
    s = str(place).lower()
    if s in ('cpu',):
        return torch.device('cpu')
    if s.startswith('gpu') or s.startswith('cuda') or s.startswith('hip') or s.startswith('xpu'):
        idx = s.split(':')[1] if ':' in s else (current_device().index if current_device().type == 'cuda' else 0)
        return torch.device('cuda', int(idx or 0))
    raise ValueError(f"unknown place {place!r}")


def set_device(device):
    """paddle.set_device('gpu:0' | 'cpu'). Returns the Place."""
    global _current
    dev = to_device(device)
    if dev.type == 'cuda':
        if not torch.cuda.is_available():
            raise ValueError("set_device('gpu') but no MI355X/HIP device is visible")
        torch.cuda.set_device(dev)
    _current = dev
    return place_of(dev)


def get_device():
    d = current_device()
    return 'cpu' if d.type == 'cpu' else f'gpu:{d.index or 0}'


def place_of(dev):
    if dev.type == 'cpu':
        return CPUPlace()
    return CUDAPlace(dev.index or 0)


def is_compiled_with_cuda():
    # ROCm build: 'cuda' in paddle's API means "the GPU backend", which is HIP here.
    return torch.cuda.is_available()


def is_compiled_with_rocm():
    return True


def is_compiled_with_xpu():
    return False


def is_compiled_with_custom_device(name=None):
    return False


def is_compiled_with_distribute():
    return True


def is_compiled_with_cinn():
    return False
