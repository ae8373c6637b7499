"""Native device allocator (csrc/alloc/allocator.cpp) behind torch's pluggable-allocator hook.

Reference: paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc and the
``FLAGS_allocator_strategy`` / ``FLAGS_auto_growth_chunk_size_in_mb`` /
``FLAGS_fraction_of_gpu_memory_to_use`` flags.  Auto-growth best-fit over large HBM chunks with
per-stream pools and neighbour coalescing; ``enable()`` must run before the process's first
device allocation (``FLAGS_use_native_allocator=1`` in the environment does it at
``import paddle``).  Once enabled, ``paddle.device.cuda.memory_allocated`` & co. report its
statistics.  A tensor used on a second stream must be kept alive until that stream is done with
it (as with ``record_stream``-free use of any stream-ordered allocator).
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_PATH = os.path.join(_HERE, '_lib', 'libpaddle_amd_alloc.so')
_state = {'lib': None, 'enabled': False}
_STAT_KEYS = ('allocated', 'reserved', 'peak_allocated', 'peak_reserved', 'num_allocs', 'num_frees',
              'num_chunks', 'num_raw_allocs', 'num_ooms')


def lib():
    """The allocator library (ctypes), loaded once."""
    if _state['lib'] is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"native allocator library missing: {LIB_PATH} (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        LL, I, P = ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p
        L.pa_alloc_config.argtypes, L.pa_alloc_config.restype = [I, LL, LL], I
        L.pa_alloc_malloc.argtypes, L.pa_alloc_malloc.restype = [LL, I, P], P
        L.pa_alloc_free.argtypes, L.pa_alloc_free.restype = [P], None
        L.pa_alloc_stats.argtypes, L.pa_alloc_stats.restype = [I, ctypes.POINTER(LL)], None
        L.pa_alloc_reset_peak.argtypes, L.pa_alloc_reset_peak.restype = [I], None
        L.pa_alloc_empty_cache.argtypes, L.pa_alloc_empty_cache.restype = [I], LL
        L.pa_alloc_largest_free.argtypes, L.pa_alloc_largest_free.restype = [I], LL
        L.pa_alloc_live_blocks.argtypes, L.pa_alloc_live_blocks.restype = [], LL
        _state['lib'] = L
    return _state['lib']


def is_enabled():
    return _state['enabled']


def enable(chunk_mb=None, fraction=None):
    """Install the native allocator as the process's device allocator.  chunk_mb: growth granule
    (FLAGS_auto_growth_chunk_size_in_mb, default 1024); fraction: cap of reserved memory as a
    fraction of the device's HBM (FLAGS_fraction_of_gpu_memory_to_use when < 1)."""
    if _state['enabled']:
        return True
    from ...framework import flags
    if chunk_mb is None:
        chunk_mb = int(flags.get_flags('FLAGS_auto_growth_chunk_size_in_mb')['FLAGS_auto_growth_chunk_size_in_mb'])
        chunk_mb = chunk_mb if chunk_mb > 0 else 1024
    limit_mb = 0
    if fraction is not None and 0 < fraction < 1 and torch.cuda.is_available():
        limit_mb = int(torch.cuda.get_device_properties(0).total_memory * fraction) >> 20
    L = lib()
    if L.pa_alloc_config(0, int(chunk_mb), int(limit_mb)) != 0:
        raise RuntimeError("native allocator: cannot reconfigure with live blocks")
    alloc = torch.cuda.memory.CUDAPluggableAllocator(LIB_PATH, 'pa_torch_alloc', 'pa_torch_free')
    try:
        torch.cuda.memory.change_current_allocator(alloc)
    except RuntimeError as e:
        raise RuntimeError("the native allocator must be enabled before the first device allocation "
                           "(set FLAGS_use_native_allocator=1 before importing paddle)") from e
    _state['enabled'] = True
    return True


def _index(device):
    if isinstance(device, torch.device):
        return device.index if device.index is not None else (torch.cuda.current_device() if device.type != 'cpu' else 0)
    if isinstance(device, str):
        return _index(torch.device(device.replace('gpu', 'cuda')))
    return int(device or 0)


def stats(device=0):
    out = (ctypes.c_longlong * 9)()
    lib().pa_alloc_stats(_index(device), out)
    return dict(zip(_STAT_KEYS, list(out)))


def empty_cache(device=0):
    """Give fully idle chunks back to the driver (after a device synchronize)."""
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return int(lib().pa_alloc_empty_cache(_index(device)))


def reset_peak(device=0):
    lib().pa_alloc_reset_peak(_index(device))


def largest_free_block(device=0):
    return int(lib().pa_alloc_largest_free(_index(device)))
