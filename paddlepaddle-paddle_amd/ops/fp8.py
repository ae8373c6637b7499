"""FP8 training path: delayed-scaling fp8 Linear (forward e4m3, gradients e5m2) on the
hand-written CDNA4 kernels.

* cast: ``csrc/fp8_cast.hip`` (``pa_fp8_cast_transpose``) — bf16 -> fp8 q and q^T in one pass,
  scale from the device-resident amax history, current amax folded in with atomics (no host
  sync anywhere on the step).
* GEMM: ``csrc/gemm.hip`` ``gemm_fp8_kernel`` (v_mfma_scale_f32_16x16x128_f8f6f4, 2x the bf16
  MFMA rate), TN layout, dequant scales read on the device.  Forward X@W, dgrad dY@W^T and wgrad
  X^T@dY are all TN GEMMs over the q / q^T images (see fp8_cast.hip's header).

Recipe (``DelayedScaling``): HYBRID = e4m3 forward operands + e5m2 gradients (the usual fp8
training recipe), E4M3 = e4m3 everywhere; ``amax_history_len`` steps of history, ``margin``
powers of two of headroom.  The first cast of a tensor seeds its history with an exact amax
pre-pass (so step 0 is scaled too).

Used by ``paddle.amp.fp8_autocast`` (dygraph: ``nn.functional.linear``) and by
``paddle.static.amp.decorate(..., use_fp8=True)`` (the Executor substitutes recorded
``addmm``/``mm``/``matmul``/``linear`` nodes whose weight is a trainable 2-D parameter).
On CPU (or for shapes outside the kernel contract) the same math runs in torch (quantise with
the same delayed scale, dequantised matmul), so the scaling logic is testable without a GPU.
"""
import contextlib
import struct
import weakref

import torch

from . import _native as N

E4M3, E5M2 = torch.float8_e4m3fn, torch.float8_e5m2
_FMT = {E4M3: 0, E5M2: 1}
_FMAX = {E4M3: 448.0, E5M2: 57344.0}


class DelayedScaling:
    """fp8 recipe (names follow the common delayed-scaling recipe)."""

    def __init__(self, margin=0, fp8_format='HYBRID', amax_history_len=16, amax_compute_algo='max'):
        fmt = str(fp8_format).upper()
        if fmt not in ('HYBRID', 'E4M3'):
            raise ValueError("fp8_format must be 'HYBRID' or 'E4M3'")
        if amax_history_len < 3:
            raise ValueError("amax_history_len must be >= 3")
        if amax_compute_algo != 'max':
            raise ValueError("only amax_compute_algo='max' is supported")
        self.margin = int(margin)
        self.fp8_format = fmt
        self.amax_history_len = int(amax_history_len)
        self.fwd_dtype = E4M3
        self.bwd_dtype = E5M2 if fmt == 'HYBRID' else E4M3

    def __repr__(self):
        return (f"DelayedScaling(margin={self.margin}, fp8_format={self.fp8_format}, "
                f"amax_history_len={self.amax_history_len})")


class FP8Meta:
    """Scaling state of one tensor role (activation / weight / gradient of one Linear)."""

    def __init__(self, dtype, history_len, margin, device):
        self.dtype = dtype
        self.L = history_len
        self.margin_mul = 2.0 ** (-margin)
        self.hist = torch.zeros(history_len, dtype=torch.float32, device=device)
        self.cur = 0
        self.calls = 0

    def scale(self):
        """Quantisation scale the next cast will use (torch mirror of the kernel's rule)."""
        L, cur = self.L, self.cur
        mask = torch.ones(L, dtype=torch.bool, device=self.hist.device)
        mask[cur] = False
        mask[(cur + 1) % L] = False
        am = self.hist[mask].max()
        s = _FMAX[self.dtype] / am * self.margin_mul
        return torch.where((am > 0) & torch.isfinite(s), s, torch.ones_like(s))

    def prep_fused(self, device):
        """Bookkeeping of a cast done inside a producer's epilogue (pa_gemm8_fp8_epi_q): returns
        (scale, amax slot, dequant scale) device tensors and advances the history like cast().
        Only once the history is seeded (the first cast measures the exact amax first)."""
        assert self.calls > 0
        L, cur = self.L, self.cur
        sc = torch.empty(1, dtype=torch.float32, device=device)
        sinv = torch.empty(1, dtype=torch.float32, device=device)
        N.check(N.lib.pa_fp8_scale_prep(N.ptr(self.hist), L, cur, _FMT[self.dtype], float(self.margin_mul), N.ptr(sc),
                                        N.ptr(sinv), N.stream()), 'fp8_scale_prep')
        slot = self.hist[cur:cur + 1]
        self.cur = (cur + 1) % L
        self.calls += 1
        return sc, slot, sinv

    def cast_weight(self, w, want_q=True, want_qt=True):
        """cast() of a weight, served from this step's batched pre-cast (begin_static_step) when
        there is one for this storage."""
        pre = self.__dict__.get('_pre')
        if pre is not None and pre[0] == _STEP[0] and pre[1] == w.data_ptr():
            return pre[2], pre[3], pre[4]
        return self.cast(w, want_q, want_qt)

    def cast(self, x2d, want_q=True, want_qt=True, colsum=None):
        """x2d: [R, C] -> (q [R,C] | None, q^T [C,R] | None, dequant scale (1-elem fp32 tensor)).
        colsum: an fp32 [R / 128 * C] buffer that also receives x2d's column sums per 128-row tile
        (the bias-gradient partials of a dY) when the HIP full-tile kernel runs; ``self.cs_done``
        tells whether it did."""
        self.cs_done = False
        x2d = x2d if x2d.dtype == torch.bfloat16 else x2d.to(torch.bfloat16)
        if x2d.stride(-1) != 1 or x2d.stride(0) % 8 or x2d.data_ptr() % 16:
            x2d = x2d.contiguous()
        R, C = x2d.shape
        L, cur = self.L, self.cur
        dev = x2d.device
        sinv = torch.empty(1, dtype=torch.float32, device=dev)
        use_hip = x2d.is_cuda and C % 8 == 0 and R > 0 and (N.lib is not None or N._load() is not None)
        if x2d.is_cuda and not use_hip and N.lib is None:
            raise RuntimeError(f"fp8 cast: HIP kernel library not loaded ({N.load_error})")
        if self.calls == 0:  # seed the history with this tensor's exact amax
            prev = (cur + L - 1) % L
            if use_hip:
                N.check(N.lib.pa_fp8_amax(N.ptr(x2d), R, C, x2d.stride(0), N.ptr(self.hist[prev:prev + 1]),
                                          N.stream()), 'fp8_amax')
            else:
                self.hist[prev] = x2d.detach().abs().max().float()
        q = torch.empty(R, C, dtype=self.dtype, device=dev) if want_q else None
        qt = torch.empty(C, R, dtype=self.dtype, device=dev) if want_qt else None
        if use_hip and colsum is not None and R % 128 == 0 and C % 128 == 0 and x2d.stride(0) % 8 == 0:
            N.check(N.lib.pa_fp8_cast_transpose_cs(N.ptr(x2d), R, C, x2d.stride(0), N.ptr(q), N.ptr(qt),
                                                   N.ptr(self.hist), L, cur, N.ptr(sinv), _FMT[self.dtype],
                                                   float(self.margin_mul), N.ptr(colsum), N.stream()),
                    'fp8_cast_transpose_cs')
            self.cs_done = True
        elif use_hip:
            N.check(N.lib.pa_fp8_cast_transpose(N.ptr(x2d), R, C, x2d.stride(0), N.ptr(q), N.ptr(qt),
                                                N.ptr(self.hist), L, cur, N.ptr(sinv), _FMT[self.dtype],
                                                float(self.margin_mul), N.stream()), 'fp8_cast_transpose')
        else:
            with torch.no_grad():
                s = self.scale()
                fm = _FMAX[self.dtype]
                qq = (x2d.float() * s).clamp(-fm, fm).to(self.dtype)
                if q is not None:
                    q.copy_(qq)
                if qt is not None:
                    qt.copy_(qq.t())
                self.hist[cur] = torch.maximum(self.hist[cur], x2d.detach().abs().max().float())
                self.hist[(cur + 1) % L] = 0.0
                sinv.copy_(1.0 / s.reshape(1))
        self.cur = (cur + 1) % L
        self.calls += 1
        return q, qt, sinv


def fp8_mm(a, b, sa, sb, bias=None, out_dtype=torch.bfloat16):
    """out[M,N] = (sa*sb) * a[M,K] @ b[N,K]^T (+ bias) with fp8 a/b (TN layout)."""
    from .gemm import hip_fp8_ok, hip_fp8_mm
    if a.is_cuda and out_dtype == torch.bfloat16 and hip_fp8_ok(a, b):
        bb = None
        if bias is not None:
            bb = bias if bias.dtype == torch.bfloat16 and bias.is_contiguous() else bias.to(torch.bfloat16).contiguous()
        return hip_fp8_mm(a, b, scale_a=sa, scale_b=sb, bias=bb)
    # outside the kernel contract (K % 128, M/N % 8) or on CPU: exact dequantised product
    out = (a.float() @ b.float().t()) * (sa * sb)
    if bias is not None:
        out = out + bias.float()
    return out.to(out_dtype)


def _colsum(dy2):
    """fp32 column sums of a bf16 [rows, N] gradient (the bias gradient) — one HIP pass, no fp32
    copy of dy (csrc/act.hip colsum) on the GPU."""
    if dy2.is_cuda and dy2.dtype in (torch.bfloat16, torch.float16):
        from . import fused
        if fused.colsum_ok(dy2):
            return fused.colsum(dy2)
    return dy2.float().sum(0)


def _slot_fp8_wgrad(a, b, sa, sb, w):
    """W.grad += sa*sb * a @ b^T by the fp8 GEMM (beta = 1) straight into w's flat gradient slot;
    False when w has no bf16 slot or the operands are outside the kernel contract."""
    from .matmul import _param_of
    from .gemm import hip_fp8_ok, hip_fp8_mm
    from ..parallel.flat_buffer import flat_grad_slot, notify_grad_ready
    p = _param_of(w) if a.is_cuda else None
    gw = flat_grad_slot(p) if p is not None else None
    if gw is None or gw.dtype != torch.bfloat16 or not gw.is_contiguous() or gw.shape != w.shape or \
            not hip_fp8_ok(a, b):
        return False
    hip_fp8_mm(a, b, scale_a=sa, scale_b=sb, out=gw, beta=1.0)
    notify_grad_ready(p)
    return True


def _slot_bias(dy2, b, part=None, nparts=0):
    from .matmul import slot_bgrad
    return b is not None and dy2.is_cuda and slot_bgrad(dy2, b, part, nparts)


class FP8State:
    """The three metas of one fp8 Linear (kept on the weight Parameter)."""

    def __init__(self, recipe, device):
        L, m = recipe.amax_history_len, recipe.margin
        self.x = FP8Meta(recipe.fwd_dtype, L, m, device)
        self.w = FP8Meta(recipe.fwd_dtype, L, m, device)
        self.g = FP8Meta(recipe.bwd_dtype, L, m, device)
        self.recipe = recipe


class _FP8Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, st):
        K, Nout = w.shape
        x2 = x.reshape(-1, K)
        need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        xq, xqt, sx = st.x.cast(x2, want_q=True, want_qt=need_dw)
        st.wref = weakref.ref(w)
        wq, wqt, sw = st.w.cast_weight(w, want_q=need_dx, want_qt=True)  # wqt: [N, K]
        y = fp8_mm(xq, wqt, sx, sw, bias=b)
        ctx.save_for_backward(xqt, wq, sx, sw)
        ctx.st, ctx.xshape, ctx.has_b, ctx.wdt, ctx.xdt = st, x.shape, b is not None, w.dtype, x.dtype
        ctx.bdt = b.dtype if b is not None else None
        ctx.w_t, ctx.b_t = w, b
        return y.reshape(*x.shape[:-1], Nout)

    @staticmethod
    def backward(ctx, dy):
        xqt, wq, sx, sw = ctx.saved_tensors
        st = ctx.st
        Nout = dy.shape[-1]
        dy2 = dy.reshape(-1, Nout)
        need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_db = ctx.has_b and ctx.needs_input_grad[2]
        M = dy2.shape[0]
        # the bias gradient's partial column sums come out of the dY cast (no second pass over dY)
        part = torch.empty((M // 128) * Nout, dtype=torch.float32, device=dy2.device) \
            if BIAS_FROM_CAST and need_db and dy2.is_cuda and M % 128 == 0 and Nout % 128 == 0 else None
        gq, gqt, sg = st.g.cast(dy2, want_q=need_dx, want_qt=need_dw, colsum=part)
        if not st.g.cs_done:
            part = None
        dx = dw = db = None
        if need_dx:
            dx = fp8_mm(gq, wq, sg, sw).reshape(ctx.xshape).to(ctx.xdt)
        if need_dw and not _slot_fp8_wgrad(xqt, gqt, sx, sg, ctx.w_t):
            dw = fp8_mm(xqt, gqt, sx, sg).to(ctx.wdt)
        if need_db:
            if part is not None:
                if not _slot_bias(dy2, ctx.b_t, part, M // 128):
                    from . import fused
                    db = fused.colsum_finish_parts(part, torch.empty(Nout, dtype=torch.float32, device=dy2.device),
                                                   M // 128, accumulate=False).to(ctx.bdt)
            elif not _slot_bias(dy2.contiguous(), ctx.b_t):
                db = _colsum(dy2).to(ctx.bdt)
        return dx, dw, db, None


def _state_for(weight_holder, w, recipe):
    st = weight_holder.__dict__.get('_fp8_state') if weight_holder is not None else None
    if st is None or st.recipe is not recipe:
        st = FP8State(recipe, w.device)
        if weight_holder is not None:
            weight_holder.__dict__['_fp8_state'] = st
    return st


_STATIC_STATES = {}
_STEP = [0]  # generation of the batched weight pre-cast (begin_static_step)


def begin_static_step():
    """Cast every weight of the static fp8 states seen so far (their q and q^T, delayed scaling
    exactly as the per-Linear cast) in ONE kernel launch per fp8 format at the start of a replay,
    instead of one small cast launch per Linear inside the step (csrc/fp8_cast.hip
    pa_fp8_cast_transpose_multi).  Weights outside the full-tile contract keep the per-call cast."""
    _STEP[0] += 1
    jobs = {}
    for st in list(_STATIC_STATES.values()):
        ref = getattr(st, 'wref', None)
        w = ref() if ref is not None else None
        m = st.w
        if (w is None or m.calls == 0 or not w.is_cuda or w.dtype != torch.bfloat16 or w.dim() != 2
                or not w.is_contiguous() or w.shape[0] % 128 or w.shape[1] % 128 or w.data_ptr() % 16):
            continue
        jobs.setdefault((w.device, _FMT[m.dtype]), []).append((m, w))
    if not jobs or (N.lib is None and N._load() is None):
        return
    for (dev, fmt), lst in jobs.items():
        blob, tile0 = bytearray(), 0
        keep = []
        for m, w in lst:
            R, C = w.shape
            q = torch.empty(R, C, dtype=m.dtype, device=dev)
            qt = torch.empty(C, R, dtype=m.dtype, device=dev)
            sinv = torch.empty(1, dtype=torch.float32, device=dev)
            blob += struct.pack('<5Qq6ifi', w.data_ptr(), q.data_ptr(), qt.data_ptr(), m.hist.data_ptr(),
                                sinv.data_ptr(), C, R, C, m.L, m.cur, C // 128, tile0, float(m.margin_mul), 0)
            tile0 += (R // 128) * (C // 128)
            m._pre = (_STEP[0], w.data_ptr(), q, qt, sinv)
            m.cur = (m.cur + 1) % m.L
            m.calls += 1
            keep.append(w)
        table = torch.frombuffer(blob, dtype=torch.uint8).pin_memory().to(dev, non_blocking=True)
        N.check(N.lib.pa_fp8_cast_transpose_multi(N.ptr(table), len(lst), tile0, fmt, N.stream()),
                'fp8_cast_transpose_multi')
        _KEEP[0] = (table, keep)  # alive until the launch has read them (the next step replaces it)


_KEEP = [None]


def fp8_linear(x, w, b=None, recipe=None, holder=None, key=None):
    """y = x @ w (+ b), w stored [in, out] (paddle layout), through the fp8 kernels."""
    recipe = recipe or _ACTIVE['recipe'] or DelayedScaling()
    if holder is None:  # static replay: state keyed by the weight storage
        st = _static_state(w, recipe, key)
    else:
        st = _state_for(holder, w, recipe)
    return _FP8Linear.apply(x, w, b, st)


def _static_state(w, recipe, key=None):
    key = key if key is not None else (id(w), w.data_ptr())
    st = _STATIC_STATES.get(key)
    if st is None or st.recipe is not recipe:
        st = _STATIC_STATES[key] = FP8State(recipe, w.device)
    return st


BIAS_FROM_CAST = True  # bias gradients from the dY cast's column sums (tests / A/B switch it)
FUSED_QUANT = True  # fp8 FFN: quantise gelu(h) / dh inside the GEMM epilogues (tests switch it)


def _fp8_epi_q(a, w, sa, sb, epi, aux, meta, bias=None):
    """(q [M,N], q^T [N,M], dequant scale) of epilogue(sa*sb * a @ w^T) quantised to meta's format
    inside the GEMM (csrc/gemm8x.hip pa_gemm8_fp8_epi_q: epi 10 gelu -> e4m3, 11 dgrad*aux ->
    e5m2), or None when the history is not seeded yet / outside the contract."""
    M, N_ = a.shape[0], w.shape[0]
    if not FUSED_QUANT or meta.calls == 0 or M % 16 or N_ % 16:
        return None
    sc, slot, sinv = meta.prep_fused(a.device)
    q = torch.empty(M, N_, dtype=meta.dtype, device=a.device)
    qt = torch.empty(N_, M, dtype=meta.dtype, device=a.device)
    N.check(N.lib.pa_gemm8_fp8_epi_q(N.ptr(a), N.ptr(w), N.ptr(q), N.ptr(qt), N.ptr(bias), N.ptr(aux), N.ptr(sa),
                                     N.ptr(sb), N.ptr(sc), N.ptr(slot), M, N_, a.shape[1], a.stride(0), w.stride(0),
                                     1.0, _FMT[a.dtype], int(epi), N.stream()), f'gemm8_fp8_epi_q{epi}')
    return q, qt, sinv


def _fp8_epi(a, w, sa, sb, epi, aux, bias=None):
    """bf16 [M, N] = epilogue(sa*sb * a @ w^T) on the fp8 GEMM (csrc/gemm8x.hip pa_gemm8_fp8_epi)."""
    M, N_ = a.shape[0], w.shape[0]
    out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
    N.check(N.lib.pa_gemm8_fp8_epi(N.ptr(a), N.ptr(w), N.ptr(out), N.ptr(bias), N.ptr(aux), N.ptr(sa), N.ptr(sb), M,
                                   N_, a.shape[1], a.stride(0), w.stride(0), out.stride(0), 1.0, _FMT[a.dtype],
                                   _FMT[w.dtype], int(epi), N.stream()), f'gemm8_fp8_epi{epi}')
    return out


class _FP8FFN(torch.autograd.Function):
    """y = gelu(x @ W1 + b1) @ W2 + b2 with both Linears in fp8 (delayed scaling, the same per-weight
    states as two fp8 Linears) and the GELU / GELU' in the fp8 GEMM epilogues: fc1 writes gelu(h)
    and gelu'(h), fc2's data gradient multiplies by gelu'(h) and reduces the fc1 bias gradient —
    the static fuse_gemm_epilogue_pass form of an fp8 feed-forward block (no activation kernels)."""

    @staticmethod
    def forward(ctx, x2, w1, b1, w2, b2, st1, st2, approximate):
        xq, xqt, sx = st1.x.cast(x2)
        st1.wref, st2.wref = weakref.ref(w1), weakref.ref(w2)
        w1q, w1qt, sw1 = st1.w.cast_weight(w1)
        h = torch.empty(x2.shape[0], w1.shape[1], dtype=torch.bfloat16, device=x2.device)
        bb1 = b1.to(torch.bfloat16).contiguous()
        fq = None if approximate else _fp8_epi_q(xq, w1qt, sx, sw1, 10, h, st2.x, bias=bb1)
        if fq is not None:  # gelu(h) leaves the fc1 GEMM already quantised (q and q^T)
            gq, gqt, sg = fq
        else:
            g = _fp8_epi(xq, w1qt, sx, sw1, 2 if approximate else 9, h, bias=bb1)
            gq, gqt, sg = st2.x.cast(g)
        w2q, w2qt, sw2 = st2.w.cast_weight(w2)
        y = fp8_mm(gq, w2qt, sg, sw2, bias=b2)
        ctx.save_for_backward(xqt, w1q, gqt, w2q, h, sx, sw1, sg, sw2)
        ctx.st = (st1, st2)
        ctx.dt = (x2.dtype, w1.dtype, b1.dtype, w2.dtype, b2.dtype)
        ctx.params = (w1, b1, w2, b2)
        return y

    @staticmethod
    def backward(ctx, dy):
        xqt, w1q, gqt, w2q, h, sx, sw1, sg, sw2 = ctx.saved_tensors
        st1, st2 = ctx.st
        xdt, w1dt, b1dt, w2dt, b2dt = ctx.dt
        dy2 = dy.contiguous()
        M = dy2.shape[0]
        N2 = dy2.shape[1]
        part2 = torch.empty((M // 128) * N2, dtype=torch.float32, device=dy2.device) \
            if BIAS_FROM_CAST and M % 128 == 0 and N2 % 128 == 0 else None
        dq, dqt, sd = st2.g.cast(dy2, colsum=part2)  # + b2's gradient partials
        if not st2.g.cs_done:
            part2 = None
        P = -(-M // 128)
        part = torch.empty(P * w2q.shape[0], dtype=torch.float32, device=dy2.device)
        fq = _fp8_epi_q(dq, w2q, sd, sw2, 11, h, st1.g, bias=part)
        if fq is not None:  # dh leaves the fc2 data-gradient GEMM already quantised (q and q^T)
            hq, hqt, shh = fq
        else:
            dh = _fp8_epi(dq, w2q, sd, sw2, 4, h, bias=part)
            hq, hqt, shh = st1.g.cast(dh)
        from . import fused
        w1, b1, w2, b2 = ctx.params
        db1 = None
        if not _slot_bias(dy2, b1, part, P):
            db1 = torch.empty(w2q.shape[0], dtype=b1dt, device=dy2.device)
            fused.colsum_finish_parts(part, db1, P, accumulate=False)
        dw2 = None if _slot_fp8_wgrad(gqt, dqt, sg, sd, w2) else fp8_mm(gqt, dqt, sg, sd).to(w2dt)
        if part2 is not None:
            db2 = None if _slot_bias(dy2, b2, part2, M // 128) else fused.colsum_finish_parts(
                part2, torch.empty(N2, dtype=torch.float32, device=dy2.device), M // 128, accumulate=False).to(b2dt)
        else:
            db2 = None if _slot_bias(dy2, b2) else _colsum(dy2).to(b2dt)
        dx = fp8_mm(hq, w1q, shh, sw1).to(xdt) if ctx.needs_input_grad[0] else None
        dw1 = None if _slot_fp8_wgrad(xqt, hqt, sx, shh, w1) else fp8_mm(xqt, hqt, sx, shh).to(w1dt)
        return dx, dw1, db1, dw2, db2, None, None, None


def ffn_ok(x2, w1, b1, w2, b2):
    """Contract of the fp8 FFN: every operand of both fp8 GEMMs and of the epilogue kernels."""
    if not (x2.is_cuda and x2.dim() == 2 and x2.dtype == torch.bfloat16 and _is_weight(w1) and _is_weight(w2)
            and eligible(x2, w1) and w2.shape[0] == w1.shape[1] and b1.dim() == 1 and b2.dim() == 1
            and b1.numel() == w1.shape[1] and b2.numel() == w2.shape[1] and x2.shape[0] % 8 == 0
            and w2.shape[1] % 8 == 0 and N._load() is not None):
        return False
    M, K, F_, N2 = x2.shape[0], x2.shape[1], w1.shape[1], w2.shape[1]
    ok = N.lib.pa_gemm8_fp8_ok
    # fc1 [M,K]x[F,K]^T, fc2 dgrad [M,N2]x[F,N2]^T; the other four go through fp8_mm's own routing
    return bool(ok(M, F_, K, K, K, F_)) and bool(ok(M, F_, N2, N2, N2, F_))


def fp8_ffn(x2, w1, b1, w2, b2, approximate=False, recipe=None):
    recipe = recipe or _STATIC_RECIPE['recipe'] or DelayedScaling()
    st1, st2 = _static_state(w1, recipe), _static_state(w2, recipe)
    return _FP8FFN.apply(x2, w1, b1, w2, b2, st1, st2, bool(approximate))


# ----------------------------------------------------------------------------- autocast state
_ACTIVE = {'enabled': False, 'recipe': None}


def fp8_enabled():
    return _ACTIVE['enabled']


@contextlib.contextmanager
def fp8_autocast(enabled=True, fp8_recipe=None):
    """Run eligible Linear layers (2-D weight, in/out features % 8) in fp8 inside the block."""
    prev = dict(_ACTIVE)
    _ACTIVE['enabled'] = bool(enabled)
    _ACTIVE['recipe'] = fp8_recipe or prev['recipe'] or DelayedScaling()
    try:
        yield
    finally:
        _ACTIVE.clear()
        _ACTIVE.update(prev)


def eligible(x, w):
    return (w.dim() == 2 and w.is_floating_point() and x.is_floating_point() and w.shape[0] % 8 == 0
            and w.shape[1] % 8 == 0 and x.shape[-1] == w.shape[0] and x.numel() > 0)


# ----------------------------------------------------------------------------- static replay
_STATIC_RECIPE = {'recipe': None}  # set by the Executor while it replays an fp8 Program


def _is_weight(w):
    return isinstance(w, torch.Tensor) and w.dim() == 2 and w.is_leaf and w.requires_grad


def _sub_addmm(orig):
    def f(bias, x, w, *a, **k):
        if not a and not k and _is_weight(w) and eligible(x, w) and bias.dim() == 1:
            return fp8_linear(x, w, bias, recipe=_STATIC_RECIPE['recipe'])
        return orig(bias, x, w, *a, **k)
    return f


def _sub_mm(orig):
    def f(x, w, *a, **k):
        if not a and not k and _is_weight(w) and eligible(x, w):
            return fp8_linear(x, w, recipe=_STATIC_RECIPE['recipe'])
        return orig(x, w, *a, **k)
    return f


def _sub_linear(orig):
    def f(x, w, bias=None):  # torch layout w [out, in]
        if _is_weight(w) and w.dim() == 2 and eligible(x, w.t()):
            return fp8_linear(x, w.t(), bias, recipe=_STATIC_RECIPE['recipe'], key=(id(w), w.data_ptr()))
        return orig(x, w, bias)
    return f


STATIC_SUBS = {
    torch.addmm: _sub_addmm(torch.addmm),
    torch.mm: _sub_mm(torch.mm),
    torch.matmul: _sub_mm(torch.matmul),
    torch.nn.functional.linear: _sub_linear(torch.nn.functional.linear),
}
