"""Embedding gather / fp32 scatter-add backward on csrc/embed_rope_optim.hip.

Reference: paddle/phi/kernels/gpu/embedding_kernel.cu, embedding_grad_kernel.cu.
"""
import torch

from . import _native as N


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w):
        idx = ids.contiguous().to(torch.int64)
        n = idx.numel()
        V, D = w.shape
        out = torch.empty(*ids.shape, D, dtype=w.dtype, device=w.device)
        N.check(N.lib.pa_embedding_fwd(N.ptr(idx), N.ptr(w), N.ptr(out), n, D, V, N.dtcode(w.dtype), N.stream()),
                'embedding_fwd')
        ctx.save_for_backward(idx)
        ctx.wshape, ctx.wdtype = (V, D), w.dtype
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
        N.check(N.lib.pa_embedding_bwd(N.ptr(idx), N.ptr(dy), N.ptr(acc), N.ptr(out), idx.numel(), D, V, 0,
                                       N.dtcode(dy.dtype), N.stream()), 'embedding_bwd')
        return None, out


def embedding(ids, w):
    if (w.shape[1] * w.element_size()) % 16 != 0 or not w.is_contiguous():
        return torch.nn.functional.embedding(ids, w)
    return _Embedding.apply(ids, w)
