"""Linear with the weight gradient accumulated IN PLACE into the flat gradient buffer.

y = x @ W + b (W: [in, out], paddle layout; with many tokens the GEMM reads a transient K-major
copy W^T from ops.gemm.kmajor_weight, the operand layout hipBLASLt runs fastest).  Backward:
  dX = dY @ W^T                                (hipBLASLt)
  W.grad += X^T @ dY                           (hand-written MFMA GEMM csrc/gemm.hip, beta = 1 epilogue)
  b.grad += colsum(dY)                         (csrc/act.hip pa_colsum, in place)
so no per-parameter gradient temporary is allocated and no separate accumulate/add kernel
runs (AccumulateGrad is bypassed; the DP/sharding engines are told the gradient is ready
through parallel.flat_buffer.notify_grad_ready).  Used only for parameters that live in flat
buffers (inside the training engines); everything else takes the ordinary autograd path.

Reference analogue: paddle/phi/kernels/fusion/gpu/fused_linear_param_grad_add_kernel.cu.
"""
import torch

from ..parallel.flat_buffer import flat_grad_slot, notify_grad_ready
from . import fused, gemm


class _LinearAccum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, box):
        if w.untyped_storage().nbytes() == 0:
            raise RuntimeError("linear weight storage is released (sharding stage-3 unit not gathered)")
        x2 = x.reshape(-1, x.shape[-1])
        wt = gemm.kmajor_weight(x2, w)  # K-major copy for the library's fast layout (transient)
        wf = w if wt is None else wt.t()
        y = torch.addmm(b, x2, wf) if b is not None else torch.mm(x2, wf)
        ctx.save_for_backward(x2, w)
        ctx.box, ctx.xshape = box, x.shape
        return y.reshape(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        wp, bp = ctx.box
        dy2 = dy.reshape(-1, dy.shape[-1])
        dx = torch.mm(dy2, w.t()).reshape(ctx.xshape) if ctx.needs_input_grad[0] else None
        gw = flat_grad_slot(wp)
        if gw is not None:
            if not gemm.wgrad_accumulate(x2, dy2, gw):
                gw.addmm_(x2.t(), dy2)
            notify_grad_ready(wp)
            dw = None
        else:
            dw = torch.mm(x2.t(), dy2)
        db = None
        if bp is not None:
            gb = flat_grad_slot(bp)
            if fused.colsum_ok(dy2):  # one column-blocked HIP pass, accumulated in place
                if gb is not None:
                    fused.colsum(dy2, gb, accumulate=True)
                    notify_grad_ready(bp)
                else:
                    db = fused.colsum(dy2).to(dy2.dtype)
            else:
                s = dy2.sum(0, dtype=torch.float32)
                if gb is not None:
                    gb.add_(s.to(gb.dtype))
                    notify_grad_ready(bp)
                else:
                    db = s.to(dy2.dtype)
        return dx, dw, db, None


def linear_accum(x, wparam, bparam):
    """x: torch tensor; wparam/bparam: paddle Parameters (flat-buffer resident)."""
    return _LinearAccum.apply(x, wparam._t, None if bparam is None else bparam._t, (wparam, bparam))


def eligible(w):
    return w._t.requires_grad and torch.is_grad_enabled() and flat_grad_slot(w) is not None
