"""Dense matmul family on the hand-written MFMA GEMM (csrc/gemm8.hip + gemm8x.hip).

Every bf16 / fp16 ``paddle.matmul`` / ``mm`` / ``bmm`` / ``@`` / two-operand ``einsum``
contraction, ``F.linear`` outside the training engines (eval, ``no_grad``, inference predictors,
layers whose weights are not in flat buffers), ``addmm``, and the static-graph / inference replay of
recorded ``torch.matmul``-family nodes lands here:

* 2-D (and N-D x 2-D with flattenable leading dims): ``gemm.mm`` — the training-step kernels for
  bf16 (decode-shaped M <= 64 on the weight-streaming skinny kernel), ``pa_gemmx`` for fp16;
* batched with broadcasting (``[..., M, K] @ [..., K, N]``): ONE launch of ``pa_gemmx`` with the
  batch on ``blockIdx.y`` and per-operand element strides (stride 0 = a broadcast operand, so a
  shared weight is never materialised per batch);
* transposes are free: each matrix is read as it sits (k-contiguous or m/n-contiguous images).

Reference: paddle/phi/kernels/impl/matmul_kernel_impl.h:960 (MatMulFunction: broadcasting, batched
strides, vector cases), python/paddle/tensor/linalg.py:177 (matmul), :2133 (bmm).  Shapes outside
the kernel contract (K % 64, odd dims, fp32, vectors, CPU / meta tensors) take torch's library path.
"""
from ..framework.flags import pa_flag  # noqa: E402
import os

import torch

from . import _native as N
from . import gemm

_DT = {torch.bfloat16: 1, torch.float16: 2}
_enabled = pa_flag('hip_matmul')


def _use(*ts):
    """All operands on the GPU, one dtype of the kernel (bf16 / fp16), HIP library on."""
    if not _enabled or not gemm._hip_gemm:
        return False
    t0 = ts[0]
    if not isinstance(t0, torch.Tensor) or t0.device.type != 'cuda' or t0.dtype not in _DT:
        return False
    for t in ts[1:]:
        if not isinstance(t, torch.Tensor) or t.device != t0.device or t.dtype != t0.dtype:
            return False
    from . import use_hip
    return use_hip(t0)


def _layout(t):
    """(trans, ld) of the last two dims: 0 = row-major (k or n contiguous), 1 = column-major."""
    r, c = t.shape[-2], t.shape[-1]
    s0, s1 = t.stride(-2), t.stride(-1)
    if s1 == 1 and (s0 >= c or r == 1):
        return 0, (s0 if r > 1 else c)
    if s0 == 1 and (s1 >= r or c == 1):
        return 1, (s1 if c > 1 else r)
    return None, None


def _bstride(t, nb):
    """Single element stride of the (collapsed) leading nb batch dims, or None when they do not
    collapse to one stride (then the operand is made contiguous)."""
    if nb == 0:
        return 0
    sizes, strides = t.shape[:nb], t.stride()[:nb]
    st = None
    # innermost non-unit batch dim sets the stride; every outer one must continue it
    expect = None
    for sz, s in zip(reversed(sizes), reversed(strides)):
        if sz == 1:
            continue
        if st is None:
            st, expect = s, s * sz
            continue
        if s != expect:
            return None
        expect = s * sz
    return 0 if st is None else st


# Per-problem choice between the hand-written kernel and the library for PLAIN GEMMs (no fused
# epilogue beyond a bias): measured once per (shape, layout, dtype) outside stream capture, the
# library taken only when it is >= 2 % faster (reference: the matmul autotune cache of
# paddle/phi/kernels/autotune/ behind paddle.incubate.autotune).  Off in multi-rank jobs, where
# replicated computations must pick the same kernel on every rank (PADDLE_AMD_GEMM_AUTOTUNE=0: off).
_TUNE = {'on': pa_flag('gemm_autotune'), 'cache': {}, 'margin': 1.02}


def _time_ms(fn, reps=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def _tune_off():
    if not _TUNE['on'] or torch.cuda.is_current_stream_capturing():
        return True
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _multi_rank():
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _tuned(key, hip_fn, lib_fn):
    """hip_fn() or lib_fn(), whichever measured faster for ``key`` (hip_fn when tuning is off or
    the problem was first seen inside a capture).  Choices measured before the job became
    multi-rank are dropped once it is (replicated computations must pick the same kernel on every
    rank); ``clear_tuning()`` resets the cache."""
    if _TUNE['cache'] and _multi_rank():
        _TUNE['cache'].clear()
    c = _TUNE['cache'].get(key)
    if c is None:
        if _tune_off():
            return hip_fn()
        th, tl = _time_ms(hip_fn), _time_ms(lib_fn)
        c = _TUNE['cache'][key] = 'lib' if tl * _TUNE['margin'] < th else 'hip'
    return hip_fn() if c == 'hip' else lib_fn()


def clear_tuning():
    """Forget every measured choice (the next call of each problem measures again)."""
    _TUNE['cache'].clear()


def tuned_choices():
    """{problem key: 'hip' | 'lib'} of the GEMM autotune cache."""
    return dict(_TUNE['cache'])


def _mm2d(a, b, bias=None, alpha=1.0):
    """a [M,K] @ b [K,N] (+ bias) for bf16 / fp16 on the hand-written kernels; None if outside."""
    if a.data_ptr() % 16 or b.data_ptr() % 16:
        return None
    if a.dtype == torch.bfloat16 and alpha == 1.0:
        if gemm._skinny_wins(a.shape[0], b.shape[1], a.shape[1]) and gemm.skinny_ok(a, b):
            return gemm.skinny_mm(a, b, bias=bias)
        if b.shape[1] < 8 and a.is_cuda:  # classifier heads: the transposed problem on the skinny kernel
            r = gemm._tiny_n(a, b, bias)
            if r is not None:
                return r
        if gemm.hip_mm_ok(a, b, 1) and (bias is None or (bias.dtype == torch.bfloat16 and bias.is_contiguous())):
            key = ('mm', a.shape, b.shape, a.stride(), b.stride(), bias is not None)
            return _tuned(key, lambda: gemm.mm(a, b, bias=bias),
                          lambda: torch.addmm(bias, a, b) if bias is not None else torch.mm(a, b))
        return None
    r = _gemmx(a.unsqueeze(0), b.unsqueeze(0), 1, bias=bias, alpha=alpha)
    return None if r is None else r[0]


def _gemmx(a3, b3, batch, bias=None, alpha=1.0, out=None, beta=0.0):
    """[batch] x (a3 [.., M, K] @ b3 [.., K, N]) in one pa_gemmx launch.  a3 / b3 carry one batch
    dim (size 1 or batch; stride 0 = broadcast).  Returns out [batch, M, N] or None."""
    ta, lda = _layout(a3)
    tb, ldb = _layout(b3)  # tb = 1: b3 is a transposed view of [N][K] (k contiguous), the kernel's transB
    if ta is None or tb is None:
        return None
    M, K = a3.shape[-2], a3.shape[-1]
    N_ = b3.shape[-1]
    if N._load() is None or not N.lib.pa_gemmx_ok(M, N_, K, lda, ldb, N_, ta, tb, _DT[a3.dtype]):
        return None
    sa = a3.stride(0) if a3.shape[0] > 1 else 0
    sb = b3.stride(0) if b3.shape[0] > 1 else 0
    if sa % 8 or sb % 8 or a3.data_ptr() % 16 or b3.data_ptr() % 16 or batch > 65535:
        return None
    if bias is not None and (bias.dtype != a3.dtype or not bias.is_contiguous() or bias.numel() != N_):
        return None
    if out is None:
        out = torch.empty(batch, M, N_, dtype=a3.dtype, device=a3.device)
        beta = 0.0
    N.check(N.lib.pa_gemmx(N.ptr(a3), N.ptr(b3), N.ptr(out), N.ptr(bias), M, N_, K, lda, ldb, N_, ta, tb, batch,
                           sa, sb, M * N_, _DT[a3.dtype], float(alpha), float(beta), N.stream()), 'gemmx')
    return out


def _matmul_raw(a, b):
    """a [..., M, K] @ b [..., K, N] (both >= 2-D, same bf16 / fp16 dtype, GPU), no autograd.
    Returns None when the shapes are outside the kernel contract."""
    K = a.shape[-1]
    if b.shape[-2] != K:
        return None
    M, N_ = a.shape[-2], b.shape[-1]
    if b.dim() == 2:
        # [..., M, K] @ [K, N]: the leading dims fold into M when they are a view
        try:
            a2 = a.view(-1, K) if a.dim() > 2 else a
        except RuntimeError:
            a2 = None
        if a2 is not None:
            y = _mm2d(a2, b)
            return None if y is None else y.view(*a.shape[:-1], N_)
    bs = torch.broadcast_shapes(a.shape[:-2], b.shape[:-2])
    nb = len(bs)
    batch = 1
    for s in bs:
        batch *= s
    if batch == 1:
        y = _mm2d(a.reshape(M, K), b.reshape(K, N_))
        return None if y is None else y.view(*bs, M, N_)
    ae = a.expand(*bs, M, K)
    be = b.expand(*bs, K, N_)
    sa, sb_ = _bstride(ae, nb), _bstride(be, nb)
    if sa is None:
        ae = ae.contiguous()
        sa = M * K
    if sb_ is None:
        be = be.contiguous()
        sb_ = K * N_
    a3 = ae.as_strided((batch if sa else 1, M, K), (sa if sa else 0, ae.stride(-2), ae.stride(-1)))
    b3 = be.as_strided((batch if sb_ else 1, K, N_), (sb_ if sb_ else 0, be.stride(-2), be.stride(-1)))
    y = _tuned(('bmm', a3.shape, b3.shape, a3.stride(), b3.stride(), a3.dtype),
               lambda: _gemmx(a3, b3, batch), lambda: torch.matmul(ae, be).reshape(batch, M, N_))
    return None if y is None else y.view(*bs, M, N_)


def _reduce_to(g, shape):
    """Sum the broadcast dims of a gradient back to ``shape``."""
    if tuple(g.shape) == tuple(shape):
        return g
    lead = g.dim() - len(shape)
    if lead > 0:
        g = g.sum(dim=tuple(range(lead)))
    dims = tuple(i for i, s in enumerate(shape) if s == 1 and g.shape[i] != 1)
    if dims:
        g = g.sum(dim=dims, keepdim=True)
    return g.reshape(shape)


def _mt(x):
    return x.transpose(-1, -2)


class _MatmulFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        y = _matmul_raw(a, b)
        if y is None:
            y = torch.matmul(a, b)
        ctx.save_for_backward(a, b)
        return y

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _reduce_to(matmul(g, _mt(b)), a.shape)
        if ctx.needs_input_grad[1]:
            if b.dim() == 2 and a.dim() > 2:
                K = a.shape[-1]
                a2 = a.reshape(-1, K)
                g2 = g.reshape(-1, g.shape[-1])
                db = matmul(a2.t(), g2)
            else:
                db = _reduce_to(matmul(_mt(a), g), b.shape)
        return da, db


def matmul(a, b):
    """torch-semantics matmul of two torch tensors on the hand-written GEMM where it applies."""
    if a.dim() < 2 or b.dim() < 2 or not _use(a, b):
        return torch.matmul(a, b)
    if torch.is_grad_enabled() and (a.requires_grad or b.requires_grad):
        return _MatmulFn.apply(a, b)
    y = _matmul_raw(a, b)
    return torch.matmul(a, b) if y is None else y


def _param_of(t):
    from ..core.tensor import _PARAMS
    p = _PARAMS.get(id(t))
    return p if p is not None and p._t is t else None


def slot_wgrad(x2, g2, w):
    """W.grad += x2^T @ g2 written by the weight-gradient GEMM (beta = 1) straight into w's flat
    gradient slot (multi-tensor optimizers keep gradients in flat buffers): no AccumulateGrad add
    pass.  False when w has no slot / the kernel contract fails (the caller returns the gradient)."""
    from ..parallel.flat_buffer import flat_grad_slot, notify_grad_ready
    p = _param_of(w)
    gw = flat_grad_slot(p) if p is not None else None
    if gw is None or gw.shape != w.shape or not gemm.wgrad_accumulate(x2, g2, gw):
        return False
    notify_grad_ready(p)
    return True


def slot_bgrad(g2, b, part=None, nparts=0):
    """b.grad += column sums of g2 (or the finish of ``nparts`` fp32 partial rows ``part``) in b's
    flat gradient slot; False when b has no slot."""
    from ..parallel.flat_buffer import flat_grad_slot, notify_grad_ready
    from . import fused
    p = _param_of(b)
    gb = flat_grad_slot(p) if p is not None else None
    if gb is None or gb.numel() != b.numel() or not gb.is_contiguous():
        return False
    if part is not None:
        fused.colsum_finish_parts(part, gb, nparts, accumulate=True)
    elif fused.colsum_ok(g2):
        fused.colsum(g2, gb, accumulate=True)
    else:
        return False
    notify_grad_ready(p)
    return True


class _LinearFn(torch.autograd.Function):
    """y = x @ W + b (W [in, out]) with all three GEMMs hand-written (the training-engine form,
    ops.linear, accumulates into flat gradient buffers; this one returns gradients)."""

    @staticmethod
    def forward(ctx, x, w, bias):
        x2 = x.reshape(-1, x.shape[-1])
        y = _mm2d(x2, w, bias=bias)
        if y is None:
            y = torch.addmm(bias, x2, w) if bias is not None else torch.mm(x2, w)
        ctx.save_for_backward(x2, w)
        ctx.xshape = x.shape
        ctx.has_bias = bias is not None
        ctx.bias_t = bias
        return y.view(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, g):
        x2, w = ctx.saved_tensors
        g2 = g.reshape(-1, g.shape[-1])
        dx = matmul(g2, w.t()).reshape(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1] and not slot_wgrad(x2, g2, w):
            dw = matmul(x2.t(), g2)
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            from . import fused
            g2c = g2.contiguous()
            if not slot_bgrad(g2c, ctx.bias_t):
                db = fused.colsum(g2c).to(g2.dtype) if fused.colsum_ok(g2c) else g2.sum(0)
        return dx, dw, db


class _FFNGeluFn(torch.autograd.Function):
    """y = gelu(x @ W1 + b1) @ W2 + b2 (W [in, out]) for static training programs (the reference's
    fuse_gemm_epilogue_pass, paddle/fluid/framework/ir/fuse_gemm_epilogue_pass.cc: linear + act
    forward and linear_grad + act_grad backward as GEMM epilogues).  fc1's epilogue writes gelu(h)
    and gelu'(h) (csrc/gemm8.hip epi 9 exact / 2 tanh); the backward's fc2 data-gradient GEMM
    multiplies by gelu'(h) in its epilogue and reduces the fc1 bias gradient there (epi 4): no
    activation kernel either way.  Returns gradients (ops.linear._MLPGelu is the flat-buffer
    form of the training engines)."""

    @staticmethod
    def forward(ctx, x2, w1, b1, w2, b2, approximate):
        from . import gemm
        h = torch.empty(x2.shape[0], w1.shape[1], dtype=x2.dtype, device=x2.device)  # gelu'(x@W1 + b1)
        g = gemm.mm_epi(x2, w1, 2 if approximate else 9, h, bias=b1)
        y = _mm2d(g, w2, bias=b2)
        if y is None:
            y = torch.addmm(b2, g, w2)
        ctx.save_for_backward(x2, w1, w2, h, g)
        ctx.biases = (b1, b2)
        return y

    @staticmethod
    def backward(ctx, dy):
        from . import gemm, fused
        x2, w1, w2, h, g = ctx.saved_tensors
        dy2 = dy.contiguous()
        M = dy2.shape[0]
        P = -(-M // 128)
        part = torch.empty(P * w2.shape[0], dtype=torch.float32, device=dy2.device)
        dh = gemm.mm_epi(dy2, w2.t(), 3, h, colsum_part=part)
        b1, b2 = ctx.biases
        db1 = None
        if not slot_bgrad(None, b1, part, P):
            db1 = torch.empty(w2.shape[0], dtype=dy2.dtype, device=dy2.device)
            fused.colsum_finish_parts(part, db1, P, accumulate=False)
        dw2 = None if slot_wgrad(g, dy2, w2) else matmul(g.t(), dy2)
        db2 = None if slot_bgrad(dy2, b2) else fused.colsum(dy2).to(dy2.dtype)
        dw1 = None if slot_wgrad(x2, dh, w1) else matmul(x2.t(), dh)
        dx = matmul(dh, w1.t()) if ctx.needs_input_grad[0] else None
        return dx, dw1, db1, dw2, db2, None


def ffn_gelu_ok(x2, w1, b1, w2, b2):
    """Contract of _FFNGeluFn: bf16 GPU operands, 2-D k-contiguous input, both biases, the fused-
    epilogue GEMM shapes of fc1 and of the fc2 data gradient."""
    from . import gemm
    ts = (x2, w1, b1, w2, b2)
    if any(not isinstance(t, torch.Tensor) or t.dtype != torch.bfloat16 or not t.is_cuda for t in ts):
        return False
    if x2.dim() != 2 or w1.dim() != 2 or w2.dim() != 2 or b1.dim() != 1 or b2.dim() != 1 or not _use(x2, w1):
        return False
    F_ = w1.shape[1]
    if x2.shape[1] != w1.shape[0] or w2.shape[0] != F_ or b1.numel() != F_ or b2.numel() != w2.shape[1]:
        return False
    if not (x2.is_contiguous() and b1.is_contiguous() and b2.is_contiguous() and w1.is_contiguous()
            and w2.is_contiguous()):
        return False
    if x2.shape[0] % 8 or F_ % 8 or w2.shape[1] % 8:
        return False
    # fc1 with its epilogue, and the fc2 data gradient dy [M, N2] @ W2^T (a transposed view) -> [M, F]
    return gemm.epi_ok(x2, w1, F_) and bool(N.lib.pa_gemm8_ok(x2.shape[0], F_, w2.shape[1], w2.shape[1], w2.shape[1],
                                                            F_, 0, 1, 1))


def ffn_gelu(x2, w1, b1, w2, b2, approximate=False):
    return _FFNGeluFn.apply(x2, w1, b1, w2, b2, bool(approximate))


_SPMD = [None]


def _spmd_on():
    """The auto-parallel SPMD mode is installed: its rules see torch ops with global-view shape
    arguments, so the Linear is issued as matmul + bias (no local-shape reshape) and stays off the
    custom-kernel Function (which the mode cannot see)."""
    m = _SPMD[0]
    if m is None:
        from ..distributed import auto_parallel_spmd as m
        _SPMD[0] = m
    return m._mode[0] is not None


def linear(x, w, bias=None):
    """paddle F.linear (W stored [in, out]) outside the training engines."""
    if _spmd_on():
        if x.dim() == 2:
            return torch.addmm(bias, x, w) if bias is not None else torch.mm(x, w)
        y = torch.matmul(x, w)
        return y + bias if bias is not None else y
    if w.dim() != 2 or x.dim() < 1 or not _use(x, w) or (bias is not None and not _use(x, bias)):
        if x.dim() == 2:
            return torch.addmm(bias, x, w) if bias is not None else torch.mm(x, w)
        if bias is not None:
            return torch.addmm(bias, x.reshape(-1, x.shape[-1]), w).reshape(*x.shape[:-1], w.shape[-1])
        return torch.matmul(x, w)
    b = bias.reshape(-1) if bias is not None else None
    if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad or (b is not None and b.requires_grad)):
        return _LinearFn.apply(x, w, b)
    x2 = x.reshape(-1, x.shape[-1])
    y = _mm2d(x2, w, bias=b)
    if y is None:
        y = torch.addmm(b, x2, w) if b is not None else torch.mm(x2, w)
    return y.view(*x.shape[:-1], w.shape[1])


def addmm(inp, x, y, beta=1.0, alpha=1.0):
    """beta * inp + alpha * (x @ y)."""
    if not _use(x, y):
        return torch.addmm(inp, x, y, beta=beta, alpha=alpha)
    if torch.is_grad_enabled() and any(t.requires_grad for t in (inp, x, y)):
        # a Linear with its bias (the recorded form of nn.Linear in static programs): all three
        # GEMMs on the hand-written kernels (ERNIE-base shapes fwd + dgrad + wgrad 1.01-1.23x the
        # library, profiles/r5c_ernie_gemm_ab.log)
        if (beta == 1.0 and alpha == 1.0 and x.dim() == 2 and y.dim() == 2 and inp.dim() == 1
                and inp.numel() == y.shape[1] and _use(x, inp)):
            return _LinearFn.apply(x, y, inp)
        return torch.addmm(inp, x, y, beta=beta, alpha=alpha)
    if x.dim() == 2 and y.dim() == 2 and inp.dtype == x.dtype and inp.is_cuda:
        if inp.dim() == 1 and inp.numel() == y.shape[1] and beta == 1.0 and alpha == 1.0:
            r = _mm2d(x, y, bias=inp.contiguous())
            if r is not None:
                return r
        # always a fresh buffer: .contiguous() of an already-contiguous [M, N] input would alias
        # the caller's tensor, and the beta-accumulating kernel writes its result in place
        out = torch.empty(x.shape[0], y.shape[1], dtype=x.dtype, device=x.device)
        out.copy_(inp.expand(x.shape[0], y.shape[1]))
        r = _gemmx(x.unsqueeze(0), y.unsqueeze(0), 1, alpha=alpha, out=out.unsqueeze(0), beta=beta)
        if r is not None:
            return out
    return torch.addmm(inp, x, y, beta=beta, alpha=alpha)


def _parse(eq, nops):
    eq = eq.replace(' ', '')
    if '.' in eq:
        return None
    if '->' in eq:
        lhs, out = eq.split('->')
    else:
        lhs = eq
        cnt = {}
        for c in lhs.replace(',', ''):
            cnt[c] = cnt.get(c, 0) + 1
        out = ''.join(sorted(c for c, n in cnt.items() if n == 1))
    ins = lhs.split(',')
    if len(ins) != nops:
        return None
    return ins, out


def einsum(eq, *operands):
    """Two-operand einsum contractions as one (batched) GEMM: operands permuted to
    [batch, free, contracted] / [batch, contracted, free] (a copy only where the labels are not
    already in that order), contracted on the hand-written kernel, result permuted to the output
    labels.  Other forms (ellipsis, repeated labels, 1 or 3+ operands) take torch.einsum."""
    if len(operands) != 2 or not _use(*operands):
        return torch.einsum(eq, *operands)
    p = _parse(eq, 2)
    if p is None:
        return torch.einsum(eq, *operands)
    (lx, ly), lo = p
    x, y = operands
    if len(set(lx)) != len(lx) or len(set(ly)) != len(ly) or len(set(lo)) != len(lo) or \
            x.dim() != len(lx) or y.dim() != len(ly) or any(c not in lx + ly for c in lo):
        return torch.einsum(eq, *operands)
    # labels summed away in only one operand: reduce them first
    sx = [i for i, c in enumerate(lx) if c not in ly and c not in lo]
    sy = [i for i, c in enumerate(ly) if c not in lx and c not in lo]
    if sx:
        x = x.sum(dim=sx)
        lx = ''.join(c for i, c in enumerate(lx) if i not in sx)
    if sy:
        y = y.sum(dim=sy)
        ly = ''.join(c for i, c in enumerate(ly) if i not in sy)
    size = {c: x.shape[i] for i, c in enumerate(lx)}
    for i, c in enumerate(ly):
        if c in size and size[c] != y.shape[i]:
            return torch.einsum(eq, *operands)
        size[c] = y.shape[i]
    bat = [c for c in lo if c in lx and c in ly]
    con = [c for c in lx if c in ly and c not in lo]
    fx = [c for c in lo if c in lx and c not in ly]
    fy = [c for c in lo if c in ly and c not in lx]
    if not con:
        return torch.einsum(eq, *operands)

    def prod(cs):
        r = 1
        for c in cs:
            r *= size[c]
        return r
    xp = x.permute(*[lx.index(c) for c in bat + fx + con]).reshape(prod(bat), prod(fx), prod(con))
    yp = y.permute(*[ly.index(c) for c in bat + con + fy]).reshape(prod(bat), prod(con), prod(fy))
    r = matmul(xp, yp).reshape(*[size[c] for c in bat + fx + fy])
    cur = bat + fx + fy
    return r.permute(*[cur.index(c) for c in lo]) if cur != list(lo) else r


def _tensor_matmul(self, other):
    return matmul(self, other)


def static_substitutions():
    """Replay-time substitutes for recorded torch GEMM nodes (static Executor, jit.load, predictor):
    the recorded program keeps plain torch targets; replay on the GPU runs them here."""
    return {torch.matmul: matmul, torch.mm: matmul, torch.bmm: matmul,
            torch.Tensor.matmul: _tensor_matmul, torch.Tensor.__matmul__: _tensor_matmul,
            torch.addmm: addmm, torch.einsum: einsum,
            torch.nn.functional.linear: lambda x, w, b=None: linear(x, w.t(), b),
            torch.nn.functional.embedding: _embedding_sub}


def _embedding_sub(*a, **k):
    from .embedding import static_embedding
    return static_embedding(*a, **k)
