"""Linear with the weight gradient accumulated IN PLACE into the flat gradient buffer.

y = x @ W + b (W: [in, out], paddle layout; with many tokens the GEMM reads a transient K-major
copy W^T from ops.gemm.kmajor_weight: both operands k-contiguous is the hand-written kernel's
fastest layout).  Every GEMM runs on the hand-written 8-phase MFMA kernel (csrc/gemm8.hip):
  y = X @ W + b                                (bias fused in the epilogue)
  dX = dY @ W^T                                (W read as it sits: k-contiguous)
  W.grad += X^T @ dY                           (beta = 1 epilogue, in place; split-K for small W)
  b.grad += colsum(dY)                         (csrc/act.hip pa_colsum, in place)
so no per-parameter gradient temporary is allocated and no separate accumulate/add kernel
runs (AccumulateGrad is bypassed; the DP/sharding engines are told the gradient is ready
through parallel.flat_buffer.notify_grad_ready).  Used only for parameters that live in flat
buffers (inside the training engines); everything else takes the ordinary autograd path.

Reference analogue: paddle/phi/kernels/fusion/gpu/fused_linear_param_grad_add_kernel.cu.
"""
from ..framework.flags import pa_flag  # noqa: E402
import os

import torch

from ..parallel.flat_buffer import (flat_grad_slot, notify_grad_ready, defer_grad, complete_deferred,
                                    register_pre_finish)
from . import fused, gemm


# Weight-gradient / data-gradient overlap: the wgrad GEMM of a Linear is launched on a side HIP
# stream right before its dgrad GEMM on the compute stream, so the two (independent) GEMMs share
# the chip; the compute stream joins the side stream before the gradient is announced ready.
# Pays where a GEMM leaves CUs idle (the QKV weight gradient: 192 256x256 tiles on 256 CUs).
WGRAD_OVERLAP = pa_flag('wgrad_overlap')
OVERLAP_MIN_TILES = 128
_side_streams = {}


def _side_stream(dev):
    s = _side_streams.get(dev)
    if s is None:
        s = _side_streams[dev] = torch.cuda.Stream(device=dev)
    return s


def _wgrad_async(x2, dy2, wp):
    """Launch W.grad += x2^T dy2 on the side stream; returns a join token, or None when the
    gradient does not live in a flat slot / overlap is off (caller uses _grad_w)."""
    if not WGRAD_OVERLAP or not x2.is_cuda:
        return None
    gw = flat_grad_slot(wp)
    if gw is None or not gemm.hip_mm_ok(x2.t(), dy2, 1) or gw.dtype != torch.bfloat16 or not gw.is_contiguous():
        return None
    # only a wgrad that leaves CUs idle in its single round of 256x256 tiles (the QKV weight
    # gradient, 192 tiles): two full-chip GEMMs side by side measured slower (cache / XCD-order
    # interference, profiles/r3_wgrad_overlap_ab.log)
    tiles = -(-gw.shape[0] // 256) * -(-gw.shape[1] // 256)
    if not (OVERLAP_MIN_TILES <= tiles < 256):
        return None
    main = torch.cuda.current_stream(x2.device)
    side = _side_stream(x2.device)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        gemm.wgrad_accumulate(x2, dy2, gw)
    x2.record_stream(side)
    dy2.record_stream(side)
    done = torch.cuda.Event()
    done.record(side)
    return done, wp


def _wgrad_join(tok):
    done, wp = tok
    torch.cuda.current_stream().wait_event(done)
    notify_grad_ready(wp)
    return None


# Grouped weight gradients: a Linear weight gradient too small to fill the chip (fewer than 128
# 256x256 tiles: the GPT out-projection, 64 tiles, which otherwise runs split-K 4 + a reduce pass) is
# deferred until the next Linear weight gradient of the same token count whose tiles complete one
# round with it (the QKV projection, 192 tiles): both then run as ONE launch of the weight-gradient
# GEMM (ops.gemm.wgrad_accumulate_grouped2).  Its grad-ready hooks are held meanwhile
# (parallel.flat_buffer.defer_grad) and anything still pending is flushed before the engines'
# end-of-backward work (register_pre_finish) or by an end-of-backward callback.
GROUP_WGRAD = pa_flag('group_wgrad')
_pending = []          # [(x2, dy2, wparam, grad slot)] — at most one deferred weight gradient
_cb_armed = [False]


def _flush_pending():
    while _pending:
        x2, dy2, wp, gw = _pending.pop()
        if not gemm.wgrad_accumulate(x2, dy2, gw):
            gw.addmm_(x2.t(), dy2)
        complete_deferred(wp)


def _end_of_backward():
    _cb_armed[0] = False
    _flush_pending()


register_pre_finish(_flush_pending)


def _grad_w_grouped(x2, dy2, wp):
    gw = flat_grad_slot(wp)
    if not GROUP_WGRAD or gw is None or not x2.is_cuda or not gemm.wgrad_grouped_ok(x2, dy2, gw):
        _flush_pending()
        return _grad_w(x2, dy2, wp)
    t = gemm.wgrad_tiles(gw)
    if _pending:
        px, pd, pw, pg = _pending[0]
        both = t + gemm.wgrad_tiles(pg)
        if px.shape[0] == x2.shape[0] and 224 <= both <= 256:
            _pending.clear()
            gemm.wgrad_accumulate_grouped2((x2, dy2, gw), (px, pd, pg))
            complete_deferred(pw)
            notify_grad_ready(wp)
            return None
        _flush_pending()
    if t < 128:
        defer_grad(wp)
        _pending.append((x2, dy2, wp, gw))
        if not _cb_armed[0]:
            _cb_armed[0] = True
            torch.autograd.Variable._execution_engine.queue_callback(_end_of_backward)
        return None
    return _grad_w(x2, dy2, wp)


class _LinearAccum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, box):
        if w.untyped_storage().nbytes() == 0:
            raise RuntimeError("linear weight storage is released (sharding stage-3 unit not gathered)")
        x2 = x.reshape(-1, x.shape[-1])
        wt = gemm.kmajor_weight(x2, w)  # transient K-major copy (the kernel's fastest layout)
        wf = w if wt is None else wt.t()
        y = gemm.mm(x2, wf, bias=b)
        ctx.save_for_backward(x2, w)
        ctx.box, ctx.xshape = box, x.shape
        return y.reshape(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        wp, bp = ctx.box
        dy2 = dy.reshape(-1, dy.shape[-1])
        tok = _wgrad_async(x2, dy2, wp)
        dx = gemm.mm(dy2, w.t()).reshape(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = _wgrad_join(tok) if tok is not None else _grad_w_grouped(x2, dy2, wp)
        db = _grad_b(dy2, bp) if bp is not None else None
        return dx, dw, db, None


def _grad_w(x2, dy2, wp):
    """W.grad += x2^T @ dy2 in the flat slot (returns None) or the gradient tensor."""
    gw = flat_grad_slot(wp)
    if gw is not None:
        if not gemm.wgrad_accumulate(x2, dy2, gw):
            gw.addmm_(x2.t(), dy2)
        notify_grad_ready(wp)
        return None
    return gemm.mm(x2.t(), dy2)


def _grad_b(dy2, bp):
    """b.grad += colsum(dy2) in the flat slot (returns None) or the gradient tensor."""
    gb = flat_grad_slot(bp)
    if fused.colsum_ok(dy2):  # one column-blocked HIP pass, accumulated in place
        if gb is not None:
            fused.colsum(dy2, gb, accumulate=True)
            notify_grad_ready(bp)
            return None
        return fused.colsum(dy2).to(dy2.dtype)
    s = dy2.sum(0, dtype=torch.float32)
    if gb is not None:
        gb.add_(s.to(gb.dtype))
        notify_grad_ready(bp)
        return None
    return s.to(dy2.dtype)


FUSE_DBIAS = True  # fc1 bias gradient from the fc2-dgrad epilogue (tests switch it)


class _MLPGelu(torch.autograd.Function):
    """y = gelu_tanh(x @ W1 + b1) @ W2 + b2 with the activation inside the GEMM epilogues:
    forward fc1 writes g = gelu(h) and gelu'(h) (h = x@W1 + b1) in one epilogue (EPI 2), backward's
    fc2 dgrad writes dh = (dy @ W2^T) * gelu'(h) (EPI 3, a plain multiply: the tanh work runs once,
    in the forward) — no standalone bias+activation kernel either way (reference:
    fusion/gpu/fused_gemm_epilogue_kernel.cu + its _grad kernel)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, boxes):
        for w in (w1, w2):
            if w.untyped_storage().nbytes() == 0:
                raise RuntimeError("linear weight storage is released (sharding stage-3 unit not gathered)")
        x2 = x.reshape(-1, x.shape[-1])
        M, F_ = x2.shape[0], w1.shape[1]
        wt1 = gemm.kmajor_weight(x2, w1)
        h = torch.empty(M, F_, dtype=x2.dtype, device=x2.device)  # gelu'(x@W1 + b1)
        g = gemm.mm_epi(x2, w1 if wt1 is None else wt1.t(), 2, h, bias=b1)
        wt2 = gemm.kmajor_weight(g, w2)
        y = gemm.mm(g, w2 if wt2 is None else wt2.t(), bias=b2)
        ctx.save_for_backward(x2, w1, w2, h, g)
        ctx.boxes, ctx.xshape = boxes, x.shape
        return y.reshape(*x.shape[:-1], w2.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, w1, w2, h, g = ctx.saved_tensors
        w1p, b1p, w2p, b2p = ctx.boxes
        dy2 = dy.reshape(-1, dy.shape[-1])
        tok2 = _wgrad_async(g, dy2, w2p)  # fc2 wgrad beside the fc2 dgrad
        dw2 = None if tok2 is not None else _grad_w(g, dy2, w2p)
        db2 = _grad_b(dy2, b2p) if b2p is not None else None
        gb1 = flat_grad_slot(b1p) if FUSE_DBIAS else None
        if gb1 is not None and gb1.is_contiguous():
            # fc1 bias gradient reduced in the fc2-dgrad GEMM epilogue (per-slab column sums of dh,
            # finished into the flat slot): no second pass over dh
            part = torch.empty(-(-dy2.shape[0] // 128) * w2.shape[0], dtype=torch.float32, device=dy2.device)
            dh = gemm.mm_epi(dy2, w2.t(), 3, h, colsum_part=part)
            fused.colsum_finish_parts(part, gb1, -(-dy2.shape[0] // 128), accumulate=True)
            notify_grad_ready(b1p)
            db1 = None
        else:
            dh = gemm.mm_epi(dy2, w2.t(), 3, h)
            db1 = _grad_b(dh, b1p)
        if tok2 is not None:
            _wgrad_join(tok2)
        tok1 = _wgrad_async(x2, dh, w1p)  # fc1 wgrad beside the fc1 dgrad
        dw1 = None if tok1 is not None else _grad_w(x2, dh, w1p)
        dx = gemm.mm(dh, w1.t()).reshape(ctx.xshape) if ctx.needs_input_grad[0] else None
        if tok1 is not None:
            _wgrad_join(tok1)
        return dx, dw1, db1, dw2, db2, None


def mlp_gelu_ok(x, w1p, b1p, w2p):
    """Fused MLP eligibility: flat-buffer params (training engines), HIP epilogue contract."""
    if b1p is None or not (eligible(w1p) and eligible(w2p) and flat_grad_slot(b1p) is not None):
        return False
    w1, w2 = w1p._t, w2p._t
    x2 = x.reshape(-1, x.shape[-1])
    return (x2.is_contiguous() and gemm.epi_ok(x2, w1, w1.shape[1]) and b1p._t.dtype == torch.bfloat16 and
            b1p._t.is_contiguous() and w2.shape[0] == w1.shape[1])


def mlp_gelu(x, w1p, b1p, w2p, b2p):
    """x: torch tensor; the four MLP parameters are paddle Parameters (flat-buffer resident)."""
    return _MLPGelu.apply(x, w1p._t, b1p._t, w2p._t, None if b2p is None else b2p._t, (w1p, b1p, w2p, b2p))


def linear_accum(x, wparam, bparam):
    """x: torch tensor; wparam/bparam: paddle Parameters (flat-buffer resident)."""
    return _LinearAccum.apply(x, wparam._t, None if bparam is None else bparam._t, (wparam, bparam))


def eligible(w):
    return w._t.requires_grad and torch.is_grad_enabled() and flat_grad_slot(w) is not None


class _TiedHead(torch.autograd.Function):
    """logits = h @ E^T for a tied [vocab, hidden] embedding E (GPT LM head), all three GEMMs on
    the hand-written kernel; E.grad accumulates in place in its flat slot (beta = 1 epilogue),
    the embedding gather's own contribution is added by autograd afterwards."""

    @staticmethod
    def forward(ctx, h, w, box):
        h2 = h.reshape(-1, h.shape[-1])
        y = gemm.mm(h2, w.t())
        ctx.save_for_backward(h2, w)
        ctx.box, ctx.hshape = box, h.shape
        return y.reshape(*h.shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dl):
        h2, w = ctx.saved_tensors
        dl2 = dl.reshape(-1, dl.shape[-1])
        dh = gemm.mm(dl2, w).reshape(ctx.hshape) if ctx.needs_input_grad[0] else None
        gw = flat_grad_slot(ctx.box)
        if gw is not None and gemm.wgrad_accumulate(dl2, h2, gw):
            notify_grad_ready(ctx.box)
            return dh, None, None
        return dh, gemm.mm(dl2.t(), h2), None


def tied_head(h, wparam):
    """h: torch [.., hidden]; wparam: the tied embedding Parameter [vocab, hidden]."""
    return _TiedHead.apply(h, wparam._t, wparam)
