"""Transformer-block fusions that also own their parameters' gradients.

* ``bias_act(x, bias_param, act)`` — y = act(x + b) with x the bias-free GEMM output.  The
  backward is ONE column-blocked kernel (csrc/act.hip ``pa_bias_act_bwd_dbias``) that writes
  dx and reduces the bias gradient from the same registers; the bias gradient is accumulated
  straight into the parameter's flat-buffer slot (no temporary, no AccumulateGrad add).
* ``dropout_add_norm(x, bias_param, residual, w, b, eps, p)`` — s = dropout(x + bias) + residual,
  y = LayerNorm/RMSNorm(s) in one pass (csrc/norm.hip ``pa_dropout_add_norm_fwd``); backward in
  one pass too: residual-stream gradient, masked input gradient, dgamma/dbeta and the bias
  gradient (reference: fused_bias_dropout_residual_layer_norm, fused_dropout_add).
* ``colsum(dy, out, accumulate)`` — bias gradient of a plain Linear (``pa_colsum``).

The dropout keep-mask is a stateless hash of (seed, offset, element), regenerated in backward.
"""
import torch

from . import _native as N
from ..parallel.flat_buffer import flat_grad_slot, notify_grad_ready

_ACTS = {'gelu': 0, 'gelu_tanh': 1, 'silu': 2, 'relu': 3, 'identity': 4}


def _slot(param, dtype=None):
    """Flat-buffer gradient slot of a paddle Parameter (None when absent or of another dtype)."""
    if param is None:
        return None
    g = flat_grad_slot(param)
    if g is None or (dtype is not None and g.dtype != dtype):
        return None
    return g


def colsum(dy2, out=None, accumulate=False):
    """Column sum of a contiguous [rows, cols] tensor in fp32 math; into ``out`` (+= when accumulate)."""
    rows, cols = dy2.shape
    if out is None:
        out = torch.empty(cols, dtype=torch.float32, device=dy2.device)
        accumulate = False
    dt = N.dtcode(dy2.dtype)
    part = torch.empty(N.lib.pa_colsum_nparts(rows, cols, dt) * cols, dtype=torch.float32, device=dy2.device)
    N.check(N.lib.pa_colsum(N.ptr(dy2), N.ptr(part), N.ptr(out), N.dtcode(out.dtype), int(bool(accumulate)), rows, cols,
                            dt, N.stream()), 'colsum')
    return out


def colsum_finish_parts(part, out, nrows, accumulate=True):
    """out (+)= the sum of the nrows fp32 partial rows in ``part`` ([nrows, cols])."""
    cols = out.numel()
    N.check(N.lib.pa_colsum_finish_parts(N.ptr(part), N.ptr(out), N.dtcode(out.dtype), int(bool(accumulate)), nrows,
                                         cols, N.stream()), 'colsum_finish_parts')
    return out


def _hip(t):
    from . import use_hip
    return use_hip(t)


def colsum_ok(dy2):
    return _hip(dy2) and dy2.dim() == 2 and dy2.is_contiguous() and dy2.dtype in (
        torch.bfloat16, torch.float16, torch.float32) and dy2.shape[1] % (16 // dy2.element_size()) == 0 and \
        N._load() is not None


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, act, box):
        x2 = x.contiguous()
        cols = x2.shape[-1]
        y = torch.empty_like(x2)
        N.check(N.lib.pa_bias_act(act, 0, None, N.ptr(x2), N.ptr(b), N.ptr(y), x2.numel(), cols, N.dtcode(x.dtype),
                                  N.stream()), 'bias_act_fwd')
        ctx.save_for_backward(x2, b)
        ctx.act, ctx.box = act, box
        return y

    @staticmethod
    def backward(ctx, dy):
        x, b = ctx.saved_tensors
        cols = x.shape[-1]
        rows = x.numel() // cols
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dt = N.dtcode(x.dtype)
        slot = _slot(ctx.box, None) if ctx.needs_input_grad[1] else None
        if ctx.needs_input_grad[1]:
            out, acc = (slot, 1) if slot is not None else (torch.empty(cols, dtype=b.dtype, device=b.device), 0)
        else:
            out, acc = torch.empty(cols, dtype=torch.float32, device=x.device), 0
        part = torch.empty(N.lib.pa_colsum_nparts(rows, cols, dt) * cols, dtype=torch.float32, device=x.device)
        N.check(N.lib.pa_bias_act_bwd_dbias(ctx.act, N.ptr(dy), N.ptr(x), N.ptr(b), N.ptr(dx), N.ptr(part), N.ptr(out),
                                            N.dtcode(out.dtype), acc, rows, cols, dt, N.stream()), 'bias_act_bwd_dbias')
        db = None
        if ctx.needs_input_grad[1]:
            if slot is not None:
                notify_grad_ready(ctx.box)
            else:
                db = out
        return dx, db, None, None


def bias_act(x, bias_param, act='gelu_tanh'):
    """act(x + bias) for a bias-free GEMM output x; bias_param is a paddle Parameter."""
    b = bias_param._t
    return _BiasAct.apply(x, b, _ACTS[act], bias_param)


def bias_act_ok(x, bias_param):
    b = bias_param._t
    return _hip(x) and b.dtype == x.dtype and x.shape[-1] % (16 // x.element_size()) == 0 and N._load() is not None


def _next_seed():
    """(seed, offset) of one dropout call, both drawn from the host generator, so paddle.seed
    fully determines every keep-mask (reference: the per-op seed/offset pair of the CUDA
    dropout kernels, derived from the paddle.seed-controlled generator)."""
    from ..device.cuda.graphs import host_rng_guard
    host_rng_guard('fused dropout + residual + norm')
    s, o = torch.randint(0, 2 ** 31 - 1, (2,), device='cpu').tolist()
    return s, o


class _DropAddNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, xb, res, w, b, eps, p, rms, boxes):
        x2, r2 = x.contiguous(), res.contiguous()
        cols = x2.shape[-1]
        rows = x2.numel() // cols
        y, s = torch.empty_like(x2), torch.empty_like(x2)
        rstd = torch.empty(rows, dtype=torch.float32, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device) if not rms else None
        seed, off = _next_seed()
        N.check(N.lib.pa_dropout_add_norm_fwd(N.ptr(x2), N.ptr(xb), N.ptr(r2), N.ptr(w), N.ptr(b), N.ptr(y), N.ptr(s),
                                              N.ptr(mean), N.ptr(rstd), rows, cols, eps, int(rms), p, seed, off,
                                              N.dtcode(x.dtype), N.dtcode(w.dtype), N.stream()), 'dropout_add_norm_fwd')
        ctx.save_for_backward(s, w, mean, rstd, xb)
        ctx.seed, ctx.off, ctx.p, ctx.rms, ctx.boxes = seed, off, p, rms, boxes
        ctx.has_b, ctx.has_xb = b is not None, xb is not None
        ctx.b_t = b
        ctx.set_materialize_grads(False)  # an unused sum output (post-LN blocks) costs no zero tensor
        return y, s

    @staticmethod
    def backward(ctx, dy, ds):
        s, w, mean, rstd, xb = ctx.saved_tensors
        cols = s.shape[-1]
        rows = s.numel() // cols
        dy = dy.contiguous() if dy is not None else torch.zeros_like(s)
        ds = ds.contiguous() if ds is not None else None
        dres, dx = torch.empty_like(s), torch.empty_like(s)
        np_ = N.lib.pa_norm_bwd_nparts(rows)
        part = torch.empty(3 * np_ * cols, dtype=torch.float32, device=s.device)
        # norm weight / bias gradients accumulate (+=) straight into their flat-buffer slots when the
        # parameters live there (no AccumulateGrad add per parameter)
        wslots = _norm_slots(w, ctx.b_t if ctx.has_b and not ctx.rms else None)
        wacc = wslots is not None
        if wacc:
            dw, db = wslots[0], wslots[1]
        else:
            dw = torch.empty_like(w)
            db = torch.empty_like(w) if ctx.has_b and not ctx.rms else None
        xb_box = ctx.boxes[0] if ctx.boxes else None
        xb_out, xb_acc, xb_slot = None, 0, None
        if ctx.has_xb and ctx.needs_input_grad[1]:
            xb_slot = _slot(xb_box)
            xb_out, xb_acc = (xb_slot, 1) if xb_slot is not None else (torch.empty_like(xb), 0)
        N.check(N.lib.pa_dropout_add_norm_bwd(N.ptr(dy), N.ptr(s), N.ptr(w), N.ptr(mean), N.ptr(rstd), N.ptr(ds),
                                              N.ptr(dres), N.ptr(dx), N.ptr(part), N.ptr(dw), N.ptr(db), N.ptr(xb_out),
                                              N.dtcode(xb_out.dtype) if xb_out is not None else 0, xb_acc, int(wacc),
                                              rows, cols, int(ctx.rms), ctx.p, ctx.seed, ctx.off, N.dtcode(s.dtype),
                                              N.dtcode(w.dtype), N.stream()), 'dropout_add_norm_bwd')
        if wacc:
            for prm in wslots[2]:
                notify_grad_ready(prm)
            dw = db = None
        dxb = None
        if xb_out is not None:
            if xb_slot is not None:
                notify_grad_ready(xb_box)
            else:
                dxb = xb_out
        return dx, dxb, dres, dw, db, None, None, None, None


SLOT_ACCUM = True  # norm weight/bias gradients into flat-buffer slots (tests switch it)


def _norm_slots(w, b):
    """(w slot, b slot or None, params) when the norm parameters' gradients live in flat buffers
    of their own dtype, else None."""
    if not SLOT_ACCUM:
        return None
    from ..core.tensor import _PARAMS
    out, prms = [], []
    for t in (w, b):
        if t is None:
            out.append(None)
            continue
        p = _PARAMS.get(id(t))
        if p is None or p._t is not t:
            return None
        g = flat_grad_slot(p)
        if g is None or g.dtype != t.dtype or not g.is_contiguous():
            return None
        out.append(g)
        prms.append(p)
    return out[0], out[1], prms


def dropout_add_norm_ok(x, w, p):
    cols = x.shape[-1]
    e = 16 // x.element_size()
    lim = 4 * 256 * e  # the fused backward keeps <= 4 vector chunks per lane
    return (_hip(x) and 0.0 < p < 1.0 and cols % e == 0 and cols <= lim and x.dtype in (torch.bfloat16, torch.float16)
            and N._load() is not None)


def dropout_add_norm(x, bias_param, residual, w, b, eps, p, rms=False):
    """(y, s): s = dropout(x + bias) + residual, y = norm(s).  bias_param: paddle Parameter or None."""
    xb = bias_param._t if bias_param is not None else None
    return _DropAddNorm.apply(x, xb, residual, w, b, eps, p, rms, (bias_param,))
