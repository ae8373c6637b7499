"""Embedding gather / fp32 scatter-add backward on csrc/embed_rope_optim.hip.

Reference: paddle/phi/kernels/gpu/embedding_kernel.cu, embedding_grad_kernel.cu.
"""
import torch

from . import _native as N


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, pad):
        idx = ids.contiguous().to(torch.int64)
        n = idx.numel()
        V, D = w.shape
        out = torch.empty(*ids.shape, D, dtype=w.dtype, device=w.device)
        N.check(N.lib.pa_embedding_fwd(N.ptr(idx), N.ptr(w), N.ptr(out), n, D, V, N.dtcode(w.dtype), N.stream()),
                'embedding_fwd')
        ctx.save_for_backward(idx)
        ctx.wshape, ctx.wdtype, ctx.pad = (V, D), w.dtype, pad
        return out

    @staticmethod
    def backward(ctx, dy):
        idx, = ctx.saved_tensors
        V, D = ctx.wshape
        dy = dy.contiguous()
        acc = torch.zeros(V, D, dtype=torch.float32, device=dy.device)
        if ctx.wdtype == torch.float32:
            out = acc
        else:
            out = torch.empty(V, D, dtype=ctx.wdtype, device=dy.device)
        N.check(N.lib.pa_embedding_bwd_pad(N.ptr(idx), N.ptr(dy), N.ptr(acc), N.ptr(out), idx.numel(), D, V, 0,
                                           ctx.pad, N.dtcode(dy.dtype), N.stream()), 'embedding_bwd')
        return None, out, None


def embedding(ids, w, padding_idx=None):
    """Gather rows of w; the gradient of the ``padding_idx`` row stays zero (torch / paddle
    semantics).  Tiny tables (token types) reduce in registers, larger ones by fp32 atomics."""
    if (w.shape[1] * w.element_size()) % 16 != 0 or not w.is_contiguous():
        return torch.nn.functional.embedding(ids, w, padding_idx)
    pad = -1 if padding_idx is None else int(padding_idx) % w.shape[0]
    return _Embedding.apply(ids, w, pad)


def static_embedding(ids, w, padding_idx=None, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, sparse=False):
    """Replay substitute of a recorded ``F.embedding`` (static Executor): the HIP gather / scatter-add
    for GPU tables, torch otherwise."""
    from . import use_hip
    if (max_norm is None and not scale_grad_by_freq and not sparse and use_hip(w) and ids.is_cuda
            and not ids.is_floating_point() and N._load() is not None):
        return embedding(ids, w, padding_idx)
    return torch.nn.functional.embedding(ids, w, padding_idx, max_norm, norm_type, scale_grad_by_freq, sparse)
