"""Channels-last batch norm (+ residual add + ReLU) on csrc/batchnorm.hip.

Reference: paddle/phi/kernels/gpu/batch_norm_kernel.cu (NHWC), fusion/gpu/fused_bn_add_activation_kernel.cu.
Training statistics are computed by the kernel (Chan-merged per-chunk mean/M2), running stats are
updated in place with paddle's momentum convention (running = m * running + (1 - m) * batch).
"""
import torch

from . import _native as N
from ..parallel.flat_buffer import flat_grad_slot, notify_grad_ready


def _ws(rows, cols, dt, dev):
    return torch.empty(N._load().pa_bn_ws_floats(rows, cols, dt), dtype=torch.float32, device=dev)


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, z, gamma, beta, run_mean, run_var, eps, momentum, training, relu, dz_sink=None):
        C = x.shape[-1]
        x2 = x.contiguous()
        rows = x2.numel() // C
        y = torch.empty_like(x2)
        z2 = z.contiguous() if z is not None else None
        dt = N.dtcode(x.dtype)
        wd = N.dtcode(gamma.dtype) if gamma is not None else 0
        if training:
            mean = torch.empty(C, dtype=torch.float32, device=x.device)
            rstd = torch.empty(C, dtype=torch.float32, device=x.device)
        else:
            mean = run_mean.float().contiguous()
            rstd = torch.rsqrt(run_var.float() + eps)
        rm = run_mean if (training and run_mean is not None and run_mean.dtype == torch.float32) else None
        rv = run_var if rm is not None else None
        parts = None
        if training and (run_mean is None or rm is not None):
            from .conv import take_bn_parts
            parts = take_bn_parts(x)  # slab statistics written by the producing conv / GEMM epilogue
        if parts is not None:
            pbuf, P, prpb = parts
            ws = torch.empty(2 * min(P, 512) * C, dtype=torch.float32, device=x.device)
            N.check(N.lib.pa_bn_fwd_parts(N.ptr(x2), N.ptr(z2), N.ptr(gamma), N.ptr(beta), N.ptr(y), N.ptr(mean),
                                          N.ptr(rstd), N.ptr(rm), N.ptr(rv), N.ptr(pbuf), P, prpb, N.ptr(ws), rows, C,
                                          float(eps), float(momentum), int(relu), dt, wd, N.stream()), 'bn_fwd_parts')
        else:
            ws = _ws(rows, C, dt, x.device)
            N.check(N.lib.pa_bn_fwd(N.ptr(x2), N.ptr(z2), N.ptr(gamma), N.ptr(beta), N.ptr(y), N.ptr(mean),
                                    N.ptr(rstd), N.ptr(rm), N.ptr(rv), N.ptr(ws), rows, C, float(eps), float(momentum),
                                    int(training), int(relu), dt, wd, N.stream()), 'bn_fwd')
        if training and run_mean is not None and rm is None:  # non-fp32 running buffers
            with torch.no_grad():
                xv = x2.reshape(rows, C).float()
                run_mean.mul_(momentum).add_(xv.mean(0).to(run_mean.dtype), alpha=1 - momentum)
                run_var.mul_(momentum).add_(xv.var(0).to(run_var.dtype), alpha=1 - momentum)
        ctx.save_for_backward(x2, y if relu else None, mean, rstd, gamma)
        ctx.relu, ctx.has_z, ctx.training = relu, z is not None, training
        ctx.has_beta = beta is not None
        ctx.dz_sink = dz_sink
        ctx.beta_t = beta
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd, gamma = ctx.saved_tensors
        if not ctx.training:
            raise RuntimeError("fused batch-norm backward with running statistics is not supported")
        C = x.shape[-1]
        rows = x.numel() // C
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dz = torch.empty_like(x) if ctx.has_z else None
        # gamma / beta gradients straight into their flat-buffer slots (accumulated in place by the
        # finishing kernel) when both parameters live in flat buffers; fresh tensors otherwise
        gs, bs, gp, bp = (_slots(gamma, ctx.beta_t) if SLOT_ACCUM and gamma is not None and ctx.has_beta
                          else (None,) * 4)
        acc = gs is not None
        dg = gs if acc else (torch.empty_like(gamma) if gamma is not None else None)
        db = bs if acc else (torch.empty_like(gamma) if (gamma is not None and ctx.has_beta) else None)
        ws = _ws(rows, C, N.dtcode(x.dtype), x.device)
        N.check(N.lib.pa_bn_bwd(N.ptr(dy), N.ptr(x), N.ptr(y), N.ptr(mean), N.ptr(rstd), N.ptr(gamma),
                                N.ptr(ctx.beta_t), N.ptr(dx),
                                N.ptr(dz), N.ptr(dg), N.ptr(db), N.ptr(ws), rows, C, int(ctx.relu), int(acc),
                                N.dtcode(x.dtype), N.dtcode(gamma.dtype) if gamma is not None else 0, N.stream()),
                'bn_bwd')
        if acc:
            notify_grad_ready(gp)
            notify_grad_ready(bp)
            dg = db = None
        if dz is not None and ctx.dz_sink is not None:
            ctx.dz_sink.buf = dz  # taken by the consuming conv's dgrad (ops/conv.py GradSink)
            dz = None
        return dx, dz, dg, db, None, None, None, None, None, None, None


SLOT_ACCUM = True  # gamma/beta gradients accumulate into flat-buffer slots in place (tests switch it)


def _slots(gamma, beta):
    """(gamma slot, beta slot, gamma param, beta param) when both parameters' gradients live in
    flat buffers with the parameters' dtype, else Nones."""
    from ..core.tensor import _PARAMS
    gp, bp = _PARAMS.get(id(gamma)), _PARAMS.get(id(beta))
    if gp is None or bp is None or gp._t is not gamma or bp._t is not beta:
        return None, None, None, None
    gs, bs = flat_grad_slot(gp), flat_grad_slot(bp)
    if gs is None or bs is None or gs.dtype != gamma.dtype or bs.dtype != beta.dtype:
        return None, None, None, None
    return gs, bs, gp, bp


def supported(x, gamma=None):
    if not x.is_cuda or x.dim() < 2 or x.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        return False
    C = x.shape[-1]
    if C % (16 // x.element_size()) != 0:
        return False
    if gamma is not None and gamma.dtype not in (torch.float32, x.dtype):
        return False
    return N._load() is not None


def channel_pad_ok(x, gamma=None):
    """The HIP kernels need C * elem_size % 16 == 0; a channel count off that grain (ShuffleNetV2's
    58/116/232) runs them on a zero-padded copy instead (``bn_nhwc_cpad``)."""
    if not x.is_cuda or x.dim() < 2 or x.dtype not in (torch.bfloat16, torch.float16, torch.float32):
        return False
    if gamma is not None and gamma.dtype not in (torch.float32, x.dtype):
        return False
    return N._load() is not None


def bn_nhwc_cpad(x, gamma, beta, run_mean, run_var, eps=1e-5, momentum=0.9, training=True):
    """batch_norm of a channels-last tensor whose channel count the kernels cannot vectorise: pad the
    channel dim to the 16-byte grain with zeros (their statistics are 0 / 0 and their outputs are
    sliced away, so gamma 1 / beta 0 there), run ``bn_act_nhwc``, slice back.  Gradients flow
    through the pad / slice; the padded running statistics are written back into the caller's."""
    C = x.shape[-1]
    v = 16 // x.element_size()
    Cp = -(-C // v) * v
    pc = Cp - C
    xp = torch.nn.functional.pad(x, (0, pc))
    gp = torch.cat([gamma, gamma.new_ones(pc)]) if gamma is not None else None
    bp = torch.cat([beta, beta.new_zeros(pc)]) if beta is not None else None
    rmp = torch.cat([run_mean, run_mean.new_zeros(pc)]) if run_mean is not None else None
    rvp = torch.cat([run_var, run_var.new_ones(pc)]) if run_var is not None else None
    y = bn_act_nhwc(xp, gp, bp, rmp, rvp, eps, momentum, training)
    if training:
        with torch.no_grad():
            if run_mean is not None:
                run_mean.copy_(rmp[:C])
            if run_var is not None:
                run_var.copy_(rvp[:C])
    return y[..., :C].contiguous()


def bn_act_nhwc(x, gamma, beta, run_mean, run_var, eps=1e-5, momentum=0.9, training=True, relu=False,
                residual=None, dz_sink=None):
    """act(batch_norm(x) [+ residual]) for a channels-last tensor (channel = last dim).  dz_sink
    (ops.conv.GradSink): hand the residual gradient to the conv that consumes the residual."""
    return _BNAct.apply(x, residual, gamma, beta, run_mean, run_var, eps, momentum, training, relu, dz_sink)
