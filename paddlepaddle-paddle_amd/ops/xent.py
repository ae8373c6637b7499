"""Fused softmax-cross-entropy (hard labels) on csrc/softmax_xent.hip.

Reference: paddle/phi/kernels/gpu/cross_entropy_kernel.cu (softmax_with_cross_entropy).
Forward reads the logits once (online logsumexp); backward writes (softmax − onehot)·dloss
directly — optionally IN PLACE over the logits buffer, so an LM head's [tokens, vocab]
logits cost one buffer for forward + backward.
"""
import torch

from . import _native as N


class _SoftmaxXent(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index, inplace_grad):
        x = logits.contiguous()
        rows, vocab = x.shape
        lab = labels.contiguous().to(torch.int64)
        loss = torch.empty(rows, dtype=torch.float32, device=x.device)
        lse = torch.empty(rows, dtype=torch.float32, device=x.device)
        N.check(N.lib.pa_xent_fwd(N.ptr(x), N.ptr(lab), N.ptr(loss), N.ptr(lse), rows, vocab, ignore_index,
                                  N.dtcode(x.dtype), N.stream()), 'xent_fwd')
        ctx.save_for_backward(x, lab, lse)
        ctx.ignore_index, ctx.inplace = ignore_index, inplace_grad
        ctx.mark_non_differentiable(lse)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        x, lab, lse = ctx.saved_tensors
        rows, vocab = x.shape
        dl = dloss.contiguous().float()
        stride = 1 if dl.numel() == rows else 0
        dx = x if ctx.inplace else torch.empty_like(x)
        N.check(N.lib.pa_xent_bwd(N.ptr(x), N.ptr(lab), N.ptr(lse), N.ptr(dl), stride, N.ptr(dx), rows, vocab,
                                  ctx.ignore_index, N.dtcode(x.dtype), N.stream()), 'xent_bwd')
        return dx, None, None, None


def softmax_cross_entropy(logits, labels, ignore_index=-100, inplace_grad=False):
    """Per-row loss (fp32) of hard-label softmax cross entropy over the last dim."""
    return _SoftmaxXent.apply(logits, labels, ignore_index, inplace_grad)
