"""HIP graph capture/replay (reference: python/paddle/device/cuda/graphs.py CUDAGraph,
cuda_graphed_layer.py).

Launch-bound inner loops (small decode steps, optimizer sweeps over many tensors) are captured
once into a hipGraph and replayed with one launch.  Inputs are copied into static buffers; all
kernels of the captured region (including this framework's ctypes-launched HIP kernels, which
launch on the current — i.e. capturing — stream) become graph nodes.
"""
import torch


def is_cuda_graph_supported():
    return torch.cuda.is_available()


class CUDAGraph:
    def __init__(self, place=None, mode="thread_local", pool_id=None):
        self._g = torch.cuda.CUDAGraph()
        self._pool = pool_id
        self._stream = None
        self._ctx = None

    def capture_begin(self):
        self._stream = torch.cuda.Stream()
        self._stream.wait_stream(torch.cuda.current_stream())
        self._ctx = torch.cuda.stream(self._stream)
        self._ctx.__enter__()
        self._g.capture_begin(pool=self._pool)

    def capture_end(self):
        self._g.capture_end()
        self._ctx.__exit__(None, None, None)
        torch.cuda.current_stream().wait_stream(self._stream)

    def replay(self):
        self._g.replay()

    def reset(self):
        self._g.reset()

    def pool(self):
        return self._g.pool()

    def print_to_dot_files(self, dirname, flags=None):
        import os
        os.makedirs(str(dirname), exist_ok=True)
        self._g.debug_dump(os.path.join(str(dirname), 'graph.dot'))


def _flatten(obj, out):
    from ...core.tensor import Tensor
    if isinstance(obj, Tensor):
        out.append(obj._t)
    elif isinstance(obj, torch.Tensor):
        out.append(obj)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _flatten(o, out)
    elif isinstance(obj, dict):
        for o in obj.values():
            _flatten(o, out)
    return out


class _Graphed:
    """Forward-only graphed callable: first ``warmup`` calls run eagerly, the next captures,
    later calls copy inputs into the static buffers and replay."""

    def __init__(self, fn, warmup=2):
        self.fn = fn
        self.warmup = warmup
        self.calls = 0
        self.graph = None
        self.static_in = None
        self.static_out = None
        self.sig = None

    def __call__(self, *args):
        from ...core.tensor import _wrap
        ins = _flatten(args, [])
        sig = tuple((t.shape, t.dtype, t.device) for t in ins)
        if self.graph is not None and sig != self.sig:
            self.graph = None  # shapes changed: recapture
            self.calls = 0
        if self.graph is None:
            self.calls += 1
            if self.calls <= self.warmup or not torch.cuda.is_available():
                return self.fn(*args)
            self.sig = sig
            self.static_in = [t.clone() for t in ins]
            it = iter(self.static_in)

            def rebuild(obj):
                from ...core.tensor import Tensor
                if isinstance(obj, Tensor):
                    return _wrap(next(it))
                if isinstance(obj, torch.Tensor):
                    return next(it)
                if isinstance(obj, (list, tuple)):
                    return type(obj)(rebuild(o) for o in obj)
                if isinstance(obj, dict):
                    return {k: rebuild(v) for k, v in obj.items()}
                return obj
            static_args = rebuild(args)
            g = CUDAGraph()
            torch.cuda.synchronize()
            g.capture_begin()
            try:
                self.static_out = self.fn(*static_args)
            finally:
                g.capture_end()
            self.graph = g
        for dst, src in zip(self.static_in, ins):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.static_out


def wrap_cuda_graph(function, mode="thread_local", memory_pool="default"):
    return _Graphed(function)
