"""ctypes binding of ``_lib/libpaddle_amd_runtime.so`` (host runtime: data-path worker pool,
prefetch queue, host event tracer — ``csrc/runtime/*.cpp``).

The library is plain C++ (no GPU code); if it is missing it is built on first use with g++
(a few seconds), so CPU-only environments get the same native data path.
"""
import ctypes
import os
import threading

_lock = threading.Lock()
_lib = None

_P, _I, _LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_LLP = ctypes.POINTER(ctypes.c_int64)
_SIGS = {
    'pa_rt_num_threads': ([], _I),
    'pa_rt_set_num_threads': ([_I], None),
    'pa_rt_gather_rows': ([_P, _LL, _LL, _P, _LL, _P], _I),
    'pa_rt_memcpy': ([_P, _P, _LL], None),
    'pa_rt_queue_new': ([_I], _P),
    'pa_rt_queue_free': ([_P], None),
    'pa_rt_queue_push': ([_P, _LL, _I], _I),
    'pa_rt_queue_pop': ([_P, _LLP, _I], _I),
    'pa_rt_queue_close': ([_P], None),
    'pa_rt_queue_size': ([_P], _I),
    'pa_rt_trace_intern': ([ctypes.c_char_p], ctypes.c_int32),
    'pa_rt_trace_name': ([ctypes.c_int32], ctypes.c_char_p),
    'pa_rt_trace_enable': ([_I], None),
    'pa_rt_trace_enabled': ([], _I),
    'pa_rt_now_ns': ([], _LL),
    'pa_rt_trace_push': ([ctypes.c_int32, ctypes.c_int32], None),
    'pa_rt_trace_pop': ([], None),
    'pa_rt_trace_record': ([ctypes.c_int32, ctypes.c_int32, _LL, _LL], None),
    'pa_rt_trace_count': ([], _LL),
    'pa_rt_trace_collect': ([_LLP, _LL], _LL),
    'pa_rt_trace_clear': ([], None),
    'pa_rt_adamw': ([_P, _P, _I, _P, _P, _P, _I, _LL] + [ctypes.c_float] * 8, _I),
}


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            import importlib.util
            here = os.path.dirname(os.path.abspath(__file__))
            spec = importlib.util.spec_from_file_location('_pa_build', os.path.join(here, '_build.py'))
            b = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(b)
            path = b.build_runtime()
            l = ctypes.CDLL(path)
            for name, (args, res) in _SIGS.items():
                f = getattr(l, name)
                f.argtypes = args
                f.restype = res
            _lib = l
    return _lib


class BlockingQueue:
    """Bounded queue of Python objects; blocking happens in C++ with the GIL released."""

    def __init__(self, capacity):
        self._l = lib()
        self._h = self._l.pa_rt_queue_new(int(capacity))
        self._objs = {}
        self._next = 0
        self._mu = threading.Lock()

    def put(self, obj, timeout=None):
        with self._mu:
            key = self._next
            self._next += 1
            self._objs[key] = obj
        r = self._l.pa_rt_queue_push(self._h, key, -1 if timeout is None else int(timeout * 1000))
        if r != 0:
            with self._mu:
                self._objs.pop(key, None)
        return r == 0

    def get(self, timeout=None):
        """Returns (ok, obj); ok False on timeout or when closed and drained."""
        v = ctypes.c_int64()
        r = self._l.pa_rt_queue_pop(self._h, ctypes.byref(v), -1 if timeout is None else int(timeout * 1000))
        if r != 0:
            return False, None
        with self._mu:
            return True, self._objs.pop(v.value)

    def close(self):
        self._l.pa_rt_queue_close(self._h)

    def size(self):
        return self._l.pa_rt_queue_size(self._h)

    def __del__(self):
        try:
            self._l.pa_rt_queue_close(self._h)
            self._l.pa_rt_queue_free(self._h)
        except Exception:
            pass


def gather_rows(src, idx, out):
    """out[i] = src[idx[i]] (numpy, C-contiguous along rows) on the native worker pool."""
    import numpy as np
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    row_bytes = src.strides[0] if src.ndim > 0 else src.itemsize
    assert src.flags['C_CONTIGUOUS'] and out.flags['C_CONTIGUOUS'] and out.shape[0] == idx.shape[0]
    r = lib().pa_rt_gather_rows(src.ctypes.data, src.shape[0], row_bytes, idx.ctypes.data, idx.shape[0],
                                out.ctypes.data)
    if r != 0:
        raise IndexError("gather_rows: index out of range")
    return out
