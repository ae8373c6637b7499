"""Fused rotary position embedding on csrc/embed_rope_optim.hip.

Reference: paddle/phi/kernels/fusion/gpu/fused_rope_kernel.cu,
python/paddle/incubate/nn/functional/fused_rotary_position_embedding.py.
cos/sin tables are built once per (seq_len, dim, base) on the host side of the device
(guide: trig tables instead of on-device sin/cos per element).
"""
import torch

from . import _native as N

_tables = {}


def rope_tables(S, D, base=10000.0, device=None):
    if device is not None and torch.device(device).type == 'meta':
        # a static program is being recorded: the tables become recorded factory + math nodes of
        # that program (replayed on its device), never a cache entry shared across programs
        inv = 1.0 / (base ** (torch.arange(0, D, 2, dtype=torch.float64, device=device) / D))
        ang = torch.arange(S, dtype=torch.float64, device=device)[:, None] * inv[None, :]
        return ang.cos().float().contiguous(), ang.sin().float().contiguous()
    key = (S, D, base, str(device))
    t = _tables.get(key)
    if t is None:
        inv = 1.0 / (base ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
        ang = torch.arange(S, dtype=torch.float64)[:, None] * inv[None, :]
        t = (ang.cos().float().to(device).contiguous(), ang.sin().float().to(device).contiguous())
        _tables[key] = t
    return t


def _launch(x, cos, sin, pos, interleaved, sign):
    B, S, H, D = x.shape
    y = torch.empty_like(x)
    N.check(N.lib.pa_rope(N.ptr(x), N.ptr(y), N.ptr(cos), N.ptr(sin), N.ptr(pos), B, S, H, D, int(interleaved), sign,
                          N.dtcode(x.dtype), N.stream()), 'rope')
    return y


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, pos, interleaved):
        x = x.contiguous()
        ctx.save_for_backward(cos, sin, pos)
        ctx.interleaved = interleaved
        return _launch(x, cos, sin, pos, interleaved, 1.0)

    @staticmethod
    def backward(ctx, dy):
        cos, sin, pos = ctx.saved_tensors
        return _launch(dy.contiguous(), cos, sin, pos, ctx.interleaved, -1.0), None, None, None, None


def apply_rope(x, cos, sin, position_ids=None, interleaved=False):
    """x: [B, S, H, D]; cos/sin: [S_max, D/2] fp32; position_ids: optional [B, S] int64."""
    pos = position_ids.contiguous().to(torch.int64) if position_ids is not None else None
    return _Rope.apply(x, cos, sin, pos, interleaved)


def rows_ok(x):
    """x: [B, S, H, D] whose (head, dim) block is contiguous and whose (b, s) rows are evenly
    strided (a contiguous tensor, or a head slice of a fused QKV projection)."""
    if x.dim() != 4 or not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        return False
    B, S, H, D = x.shape
    if N.lib is None and N._load() is None:
        return False
    return (D % 16 == 0 and x.stride(3) == 1 and x.stride(2) == D and x.stride(0) == S * x.stride(1)
            and x.stride(1) % 8 == 0 and x.data_ptr() % 16 == 0)


def rope_rows(x, y, cos, sin, pos=None, interleaved=False, sign=1.0):
    """y = rope(x) (sign -1: the inverse rotation) over strided rows (``rows_ok`` layouts; y may
    be x: in place) on csrc/embed_rope_optim.hip pa_rope_rows (8 rotation pairs per work item)."""
    B, S, H, D = x.shape
    lib = N.lib if N.lib is not None else N._load()
    N.check(lib.pa_rope_rows(N.ptr(x), x.stride(1), N.ptr(y), y.stride(1), N.ptr(cos), N.ptr(sin), N.ptr(pos),
                               B, S, H, D, int(interleaved), float(sign), N.dtcode(x.dtype), N.stream()), 'rope_rows')
    return y
