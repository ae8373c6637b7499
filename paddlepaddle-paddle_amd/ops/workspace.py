"""Per-device scratch workspaces shared by kernel launches (flash-attention dS^T, weight-only GEMM
split-K partials, ...), safe under HIP-graph capture.

A workspace grows when a larger shape arrives.  A buffer that was ever handed to a launch while a
stream was capturing is baked into that graph's kernel arguments, so when it is superseded it is
retained (never returned to the allocator) for as long as the process lives — a later replay then
still writes into memory nobody else owns.  Buffers never seen by a capture are simply dropped.
``release()`` frees every buffer no graph has captured (e.g. after a long-sequence eval pass) and
``limit_bytes`` bounds a workspace: callers take their no-workspace fallback above it.

Reference analogue: the workspace handling of paddle/phi/kernels/gpu/flash_attn_grad_kernel.cu
(a per-call DenseTensor from the allocator; a caching allocator keeps it around).
"""
import torch


class Workspace:
    def __init__(self, name, limit_bytes=None):
        self.name = name
        self.limit_bytes = limit_bytes
        self._cur = {}       # (device, dtype) -> [tensor, captured]
        self._retained = []  # superseded buffers some captured graph may still address

    def fits(self, numel, dtype):
        if self.limit_bytes is None:
            return True
        return numel * torch.empty((), dtype=dtype).element_size() <= self.limit_bytes

    def get(self, numel, dtype, device, min_numel=0):
        key = (str(device), dtype)
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        ent = self._cur.get(key)
        if ent is None or ent[0].numel() < numel:
            if ent is not None and ent[1]:
                self._retained.append(ent[0])
            ent = [torch.empty(max(int(numel), int(min_numel)), dtype=dtype, device=device), False]
            self._cur[key] = ent
        if capturing:
            ent[1] = True
        return ent[0]

    def release(self):
        """Drop every buffer no captured graph addresses; returns the number of bytes released."""
        freed = 0
        for key, ent in list(self._cur.items()):
            if not ent[1]:
                freed += ent[0].numel() * ent[0].element_size()
                del self._cur[key]
        return freed

    def nbytes(self):
        return sum(e[0].numel() * e[0].element_size() for e in self._cur.values()) + \
            sum(t.numel() * t.element_size() for t in self._retained)


_ALL = []


def workspace(name, limit_bytes=None):
    w = Workspace(name, limit_bytes)
    _ALL.append(w)
    return w


def release_all():
    """Release every uncaptured kernel workspace (paddle.device.cuda.empty_cache calls this)."""
    return sum(w.release() for w in _ALL)
