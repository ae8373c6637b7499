"""NHWC conv2d on hand-written implicit-GEMM MFMA kernels (csrc/conv.hip), forward and backward.

Reference: paddle/phi/kernels/gpudnn/conv_kernel.cu (forward), conv_grad_kernel.cu (backward).
* Forward: im2col folded into the LDS-DMA source addresses, zero padding via a zero block, bias
  fused; the weight is packed into the [Cout][R][S][C] k-contiguous image the kernel stages
  (re-packed per call).  Needs C % 32 == 0; the 3-channel RGB stem forward stays on the storage
  layer's direct convolution (an explicit im2col + 1x1 MFMA path, pa_im2col_nhwc, is available
  as conv2d_fwd_im2col but measured slower there).
* Batch-norm statistics (fused_bn_stats): the forward epilogue can also emit per-slab channel
  (mean, M2) for the batch norm that consumes the output (ops/batchnorm.py).
* Data gradient (any stride): stride classes of input pixels, each a stride-1 implicit GEMM over
  dY with the taps that reach it, all classes in one launch (pa_conv2d_dgrad_classes).
* Filter gradient (any R x S / stride / padding): implicit GEMM with the pixels as the reduction
  axis, split over the grid (pa_conv2d_wgrad); inputs with C % 8 != 0 (the stem) are zero-padded
  to 8 channels for it.
* 1x1 stride-1 convolutions with wide channel counts: plain GEMMs on the 8-phase MFMA GEMM
  (forward, data gradient, filter gradient), where measured faster (_pointwise).
The storage layer's convolution backward (MIOpen) remains only as the fallback for shapes the
kernels reject (grouped / odd channel counts) or when PADDLE_AMD_HIP_CONV_BWD=0.
"""
from ..framework.flags import pa_flag  # noqa: E402
import os

import torch

from . import _native as N
from ..parallel.flat_buffer import flat_grad_slot, notify_grad_ready


SLOT_ACCUM = True  # filter gradients accumulate into flat-buffer slots in place (tests switch it)


def _param_of(t):
    """The paddle Parameter whose storage tensor is ``t`` (None for plain tensors)."""
    from ..core.tensor import _PARAMS
    p = _PARAMS.get(id(t))
    return p if p is not None and p._t is t else None

_enabled = pa_flag('hip_conv')
_bwd_enabled = pa_flag('hip_conv_bwd')
_wgrad_hip = pa_flag('hip_conv_wgrad')


def supported(x, w, groups):
    """The conv runs through _Conv2dNHWC: a hand-written forward, or (small C, e.g. the RGB stem)
    the library forward with the hand-written backward."""
    if not _enabled or groups != 1 or x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        return False
    if x.dim() != 4 or w.dim() != 4 or not x.is_cuda:
        return False
    if N.lib is None and N._load() is None:
        return False
    Cout, C, R, S = w.shape
    if x.shape[3] != C:
        return False
    return bool(N.lib.pa_conv2d_fwd_ok(C, Cout, R, S)) or (_bwd_enabled and Cout % 8 == 0 and C < 8)


def fwd_ok(w):
    Cout, C, R, S = w.shape
    return bool(N.lib.pa_conv2d_fwd_ok(C, Cout, R, S))


def _packed(w):
    """[Cout][R][S][C] image of an OIHW filter.  Re-packed on every call: the fused optimizer
    kernels update parameters in place through raw pointers, which does not bump the tensor
    version counter, so no cache keyed on the tensor could tell a stale image (one small copy
    per conv per step)."""
    return w.detach().permute(0, 2, 3, 1).contiguous()


def _out_hw(H, W, R, S, stride, pad, dil):
    return ((H + 2 * pad[0] - dil[0] * (R - 1) - 1) // stride[0] + 1,
            (W + 2 * pad[1] - dil[1] * (S - 1) - 1) // stride[1] + 1)


# ---- batch-norm statistics from the convolution epilogue (fused_bn statistics)
# Inside ``fused_bn_stats()`` (the ResNet forward), every forward convolution without bias that runs
# on a hand-written kernel also writes the per-channel (mean, M2) of each 64-256-row slab of its
# output (csrc/conv.hip pa_conv2d_fwd_stats, csrc/gemm8.hip epi 5).  The training batch norm that
# consumes that output (ops/batchnorm.py) takes them instead of re-reading the activation for its
# statistics pass.  Entries are keyed by the output tensor object (weak reference) and popped by
# the consumer.
_stats_mode = [0]
# (data_ptr, numel) of y -> (y, parts [2][P][C] fp32, P, rows per slab, y._version).  y is held
# strongly, for the fused_bn_stats() scope only: a weak reference died with the NHWC tensor object
# when an NCHW conv2d handed back only its permuted view, and its norm then recomputed statistics
_bn_parts = {}


class fused_bn_stats:
    """Context: forward convolutions also emit batch-norm slab statistics of their outputs."""

    def __enter__(self):
        _stats_mode[0] += 1
        return self

    def __exit__(self, *exc):
        _stats_mode[0] -= 1
        if _stats_mode[0] == 0:
            _bn_parts.clear()
        return False


def _want_stats(b):
    return _stats_mode[0] > 0 and b is None and _stats_enabled


_stats_enabled = pa_flag('conv_bn_stats')


def _parts_key(t):
    # keyed by memory, not by tensor object: an NCHW conv2d returns its NHWC output as a permuted
    # view (ops reached through nn.functional see a different tensor object with the same storage)
    return (t.data_ptr(), t.numel())


def _stash_parts(y, parts, P, rpb):
    _bn_parts[_parts_key(y)] = (y, parts, P, rpb, y._version)


def take_bn_parts(x):
    """(parts, P, rows per slab) of a tensor produced under fused_bn_stats() (or a view of it with
    the same memory), or None."""
    e = _bn_parts.pop(_parts_key(x), None)
    if e is None:
        return None
    if x._version != e[4] or x.shape[-1] != e[0].shape[-1]:
        # modified in place since the epilogue wrote them (views share the version counter), or
        # another channel view of the same memory
        return None
    return e[1], e[2], e[3]


def _fwd_packed(x, wpk, b, stride, pad, dil):
    """x: [N,H,W,C] bf16, wpk: packed [Cout][R][S][C] -> y [N,Ho,Wo,Cout]."""
    x = x.contiguous()
    Nb, H, W, C = x.shape
    Cout, R, S, _ = wpk.shape
    Ho, Wo = _out_hw(H, W, R, S, stride, pad, dil)
    Cp = int(N.lib.pa_conv2d_fwd_cpad(C))
    if Cp != C:  # C % 32 != 0: zero filter channels up to the padded K decomposition
        wpk = torch.cat([wpk, wpk.new_zeros(Cout, R, S, Cp - C)], 3)
    pt = int(N.lib.pa_conv2d_fwd_pad_taps(Cp, R, S))
    if pt:  # K = taps * C made a multiple of 64 with zero taps (e.g. 3x3 over 32 channels)
        wpk = torch.cat([wpk.reshape(Cout, R * S * Cp), wpk.new_zeros(Cout, pt * Cp)], 1)
    y = torch.empty(Nb, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    if _want_stats(b):
        rpb = int(N.lib.pa_conv2d_fwd_stat_rows(Cout))
        P = -(-(Nb * Ho * Wo) // rpb)
        parts = torch.empty(2 * P * Cout, dtype=torch.float32, device=x.device)
        N.check(N.lib.pa_conv2d_fwd_stats(N.ptr(x), N.ptr(wpk), N.ptr(y), N.ptr(parts), Nb, H, W, C, Cout, R, S,
                                          stride[0], stride[1], pad[0], pad[1], dil[0], dil[1], Ho, Wo, N.stream()),
                'conv2d_fwd_stats')
        _stash_parts(y, parts, P, rpb)
        return y
    bb = b.to(torch.bfloat16).contiguous() if b is not None else None
    N.check(N.lib.pa_conv2d_fwd(N.ptr(x), N.ptr(wpk), N.ptr(y), N.ptr(bb), Nb, H, W, C, Cout, R, S, stride[0],
                                stride[1], pad[0], pad[1], dil[0], dil[1], Ho, Wo, N.stream()), 'conv2d_fwd')
    return y


def conv2d_fwd(x, w, b, stride, pad, dil):
    """x: [N,H,W,C] bf16 (NHWC), w: [Cout,C,R,S] (paddle OIHW) -> y [N,Ho,Wo,Cout]."""
    return _fwd_packed(x, _packed(w), b, stride, pad, dil)


# Not routed: on the ResNet50 stem (256 x 224 x 224 x 3, 7x7/2) the im2col matrix is [3.2M, 192]
# = 1.23 GB written and read back; im2col 0.54 ms + the 1x1 conv 0.12 ms lose to the library's
# direct convolution (0.36 ms, profiles/r3s3_im2col_ab.log), and the stem kernel
# (csrc/conv_stem.hip, 0.22 ms) replaced both.  Kept as an explicit API for few-channel convs.
def conv2d_fwd_im2col(x, w, b, stride, pad, dil):
    """y = conv(x, w) as im2col(x) [M, Kp] times the [Cout][Kp] filter image, the second step a
    1 x 1 convolution on conv_fwd_kernel (so the batch-norm statistics epilogue applies as for
    any other forward).  k = r * RK + s * C + c (RK = S*C rounded up to 8: each filter row one
    contiguous input run and one aligned output run), Kp = R*RK rounded up to 64, zero slots."""
    x = x.contiguous()
    Nb, H, W, C = x.shape
    Cout, _, R, S = w.shape
    Ho, Wo = _out_hw(H, W, R, S, stride, pad, dil)
    RK = -(-(S * C) // 8) * 8
    Kp = -(-(R * RK) // 64) * 64
    M = Nb * Ho * Wo
    cols = torch.empty(M, Kp, dtype=torch.bfloat16, device=x.device)
    N.check(N.lib.pa_im2col_nhwc(N.ptr(x), N.ptr(cols), Nb, H, W, C, R, S, stride[0], stride[1], pad[0], pad[1],
                                 dil[0], dil[1], Ho, Wo, Kp, N.stream()), 'im2col_nhwc')
    wimg = torch.zeros(Cout, R, RK, dtype=torch.bfloat16, device=x.device)
    wimg[:, :, :S * C] = w.detach().permute(0, 2, 3, 1).reshape(Cout, R, S * C)
    wpk = torch.zeros(Cout, 1, 1, Kp, dtype=torch.bfloat16, device=x.device)
    wpk[:, 0, 0, :R * RK] = wimg.reshape(Cout, R * RK)
    y4 = _fwd_packed(cols.view(1, M, 1, Kp), wpk, b, (1, 1), (0, 0), (1, 1))
    y = y4.view(Nb, Ho, Wo, Cout)
    e = take_bn_parts(y4)
    if e is not None:  # statistics were stashed under the [1, M, 1, Cout] output: re-key them to y
        _stash_parts(y, *e[:3])
    return y


def conv2d_dgrad(dy, w, x_hw, pad, dil):
    """Stride-1 data gradient as a forward conv of dy with the spatially flipped, transposed
    filter ([C][R][S][Cout] image) and padding dil*(R-1) - pad (same kernel as the forward)."""
    Cout, C, R, S = w.shape
    wpk = w.detach().flip(2, 3).permute(1, 2, 3, 0).contiguous()
    p2 = (dil[0] * (R - 1) - pad[0], dil[1] * (S - 1) - pad[1])
    if p2[0] < 0 or p2[1] < 0:
        return None
    gx = _fwd_packed(dy, wpk, None, (1, 1), p2, dil)
    return gx if tuple(gx.shape[1:3]) == tuple(x_hw) else None


_DGRAD_PLANS = {}


def _dgrad_plan(w_shape, x_hw, stride, pad, dil, device):
    """Stride classes of a data gradient (cached per geometry): ((a, b, T) per class, tap order,
    dY offsets, whether some input pixels get no tap (zero fill))."""
    import ctypes
    key = (tuple(w_shape), tuple(x_hw), tuple(stride), tuple(pad), tuple(dil), str(device))
    plan = _DGRAD_PLANS.get(key)
    if plan is not None:
        return plan
    Cout, C, R, S = w_shape
    H, W = x_hw
    sh, sw = stride
    classes, empty = [], False
    for a in range(sh):
        for b in range(sw):
            if H - a <= 0 or W - b <= 0:
                continue
            taps = [(r * S + q, (a + pad[0] - r * dil[0]) // sh, (b + pad[1] - q * dil[1]) // sw)
                    for r in range(R) if (a + pad[0] - r * dil[0]) % sh == 0
                    for q in range(S) if (b + pad[1] - q * dil[1]) % sw == 0]
            if taps:
                classes.append((a, b, taps))
            else:
                empty = True
    # a class whose K = taps * Cout is an odd multiple of 32 gets a zero tap (filter slot R*S holds
    # zeros; its dY offset lies far outside, so the kernel reads the zero block)
    classes = [(a, b, taps + ([(R * S, -30000, -30000)] if (len(taps) * Cout) % 64 else []))
               for a, b, taps in classes]
    flat = [t for _, _, taps in classes for t in taps]
    ok = (0 < len(classes) <= 9 and len(flat) <= 64 and Cout % 32 == 0 and C % 8 == 0 and H < 16384 and W < 16384
          and all((len(t) * Cout) % 64 == 0 for _, _, t in classes))
    order = [t[0] for t in flat]
    idx = None if order == list(range(R * S)) else torch.tensor(order, device=device)
    cls = (ctypes.c_int * (3 * max(1, len(classes))))(*[v for a, b, taps in classes for v in (a, b, len(taps))])
    th = (ctypes.c_int * max(1, len(flat)))(*[t[1] for t in flat])
    tw = (ctypes.c_int * max(1, len(flat)))(*[t[2] for t in flat])
    plan = (ok, len(classes), idx, empty, cls, th, tw, R * S in order)
    _DGRAD_PLANS[key] = plan
    return plan


def conv2d_dgrad_classes(dy, w, x_hw, stride, pad, dil):
    """Data gradient of any stride: dX splits into stride_h x stride_w classes of input pixels
    (ih = a + s_h*i, iw = b + s_w*j); each class only sees the filter taps with
    (a + pad - r*dil) % s == 0, at dY offset (a + pad - r*dil) / s — a stride-1 implicit GEMM over dY
    with a subset of taps whose output lands on every s-th pixel; all classes run in one launch
    (csrc/conv.hip pa_conv2d_dgrad_classes).  Stride 1 is the single class with every tap."""
    import ctypes
    Cout, C, R, S = w.shape
    H, W = x_hw
    ok, ncls, idx, empty, cls, th, tw, zpad = _dgrad_plan(w.shape, x_hw, stride, pad, dil, dy.device)
    if not ok:
        return None
    dy = dy.contiguous()
    Nb, Hd, Wd, _ = dy.shape
    wt = w.detach().to(torch.bfloat16).permute(1, 2, 3, 0).reshape(C, R * S, Cout)
    if zpad:  # zero-tap slot
        wt = torch.cat([wt, wt.new_zeros(C, 1, Cout)], 1)
    wd = (wt if idx is None else wt.index_select(1, idx)).contiguous()  # [C][taps in class order][Cout]
    dx = (torch.zeros if empty else torch.empty)(Nb, H, W, C, dtype=torch.bfloat16, device=dy.device)
    vp = lambda arr: ctypes.cast(arr, ctypes.c_void_p)  # noqa: E731
    N.check(N.lib.pa_conv2d_dgrad_classes(N.ptr(dy), N.ptr(wd), N.ptr(dx), Nb, Hd, Wd, Cout, C, H, W, stride[0],
                                          stride[1], ncls, vp(cls), vp(th), vp(tw), N.stream()),
            'conv2d_dgrad_classes')
    return dx


def conv2d_wgrad_1x1(dy, x, out=None):
    """1x1 / stride-1 / no-padding filter gradient: dW[co, c] = sum_pixels dY[p, co] X[p, c] on the
    hand-written GEMM (A = dY^T read with tr_b16; split-K over pixels when the output is small).
    out: bf16 [Cout, C, 1, 1] slot accumulated in place (beta = 1)."""
    from . import gemm
    Cout, C = dy.shape[-1], x.shape[-1]
    dy2, x2 = dy.reshape(-1, Cout), x.reshape(-1, C)
    a = dy2.t()
    tiles = -(-Cout // 256) * -(-C // 256)
    sk = 1
    while sk * 2 * tiles <= 256 and dy2.shape[0] % (64 * sk * 2) == 0:
        sk *= 2
    if not gemm.hip_mm_ok(a, x2, sk):
        return None
    if out is not None:
        return gemm.hip_mm(a, x2, out=out.view(Cout, C), beta=1.0, splitk=sk).view(Cout, C, 1, 1)
    return gemm.hip_mm(a, x2, splitk=sk).view(Cout, C, 1, 1)


_WGRAD_TARGET_BLOCKS = 512  # two waves of 256 CUs over (tiles x pixel splits)


def wgrad_ok(x, w):
    Cout, C = w.shape[0], w.shape[1]
    return _bwd_enabled and bool(N.lib.pa_conv2d_wgrad_ok(C, Cout))


def conv2d_wgrad(dy, x, w_shape, stride, pad, dil, out=None):
    """Filter gradient of any R x S / stride / padding / dilation on the implicit-GEMM kernel
    (pixels are the reduction axis, split over the grid; fp32 slabs folded into the OIHW bf16
    gradient by a second kernel).  out: a bf16 [Cout, C, R, S] gradient slot the result is
    ACCUMULATED into (returned); None -> a fresh tensor."""
    Cout, C, R, S = w_shape
    x, dy = x.contiguous(), dy.contiguous()
    if R == S == 1 and tuple(stride) == (1, 1) and tuple(pad) == (0, 0) and C < Cout and Cout % 8 == 0:
        if out is not None:
            return None  # transposed form below: the caller accumulates
        # 1x1: dW = dY^T X is symmetric in (X, dY) — put the wider channel count on the 256-wide
        # tile side (a 64-channel input would leave 3/4 of every 256-row tile empty)
        return conv2d_wgrad(x, dy, (C, Cout, 1, 1), stride, pad, dil).view(C, Cout).t().contiguous().view(Cout, C, 1, 1)
    Nb, H, W, _ = x.shape
    _, Ho, Wo, _ = dy.shape
    M = R * S * C
    bn = 64 if Cout <= 64 else 128
    tiles = -(-M // 256) * -(-Cout // bn)
    P = Nb * Ho * Wo
    want = max(1, min(_WGRAD_TARGET_BLOCKS // tiles, P // 512))
    splits = int(N.lib.pa_conv2d_wgrad_splits(Nb, Ho, Wo, want))
    ws = torch.empty((splits + -(-splits // 16)) * M * Cout, dtype=torch.float32, device=x.device)
    acc = out is not None
    dw = out if acc else torch.empty(Cout, C, R, S, dtype=torch.bfloat16, device=x.device)
    N.check(N.lib.pa_conv2d_wgrad(N.ptr(x), N.ptr(dy), N.ptr(ws), N.ptr(dw), Nb, H, W, C, Cout, R, S, stride[0],
                                  stride[1], pad[0], pad[1], dil[0], dil[1], Ho, Wo, want, int(acc), N.stream()),
            'conv2d_wgrad')
    return dw


# 1x1 / stride-1 / unpadded convolutions are plain GEMMs over the N*H*W pixel rows; the 8-phase MFMA
# GEMM (csrc/gemm8.hip) runs them faster than the implicit-GEMM conv kernel once the GEMM's N side
# fills its 256-wide tiles (tools/conv1x1_gemm_bench.py, profiles/r2_conv1x1_gemm.log: forward when
# Cout >= 128, data gradient when C >= 128, filter gradient when C >= 512 and Cout >= C / 2).
_gemm_1x1 = pa_flag('conv1x1_gemm')


def _pointwise(w, stride, pad, dil):
    return (_gemm_1x1 and w.shape[2] == 1 and w.shape[3] == 1 and tuple(stride) == (1, 1)
            and tuple(pad) == (0, 0))


def _gemm_fwd_1x1(x, w, b):
    from . import gemm
    Cout, C = w.shape[0], w.shape[1]
    if Cout < 128:
        return None
    x2 = x.contiguous().view(-1, C)
    wt = w.detach().view(Cout, C).t()  # [C, Cout] view of the k-contiguous [Cout][C] filter
    bb = b.to(torch.bfloat16).contiguous() if b is not None else None
    if not gemm.hip_mm_ok(x2, wt):
        return None
    if _want_stats(b) and gemm.epi_ok(x2, wt, Cout):
        y, parts, P = gemm.mm_bn_stats(x2, wt)
        y = y.view(*x.shape[:3], Cout)
        _stash_parts(y, parts, P, 128)
        return y
    return gemm.hip_mm(x2, wt, bias=bb).view(*x.shape[:3], Cout)


def _gemm_dgrad_1x1(dy, w, acc=None):
    """dX = dY @ W (+ acc, accumulated in place by the beta = 1 epilogue)."""
    from . import gemm
    Cout, C = w.shape[0], w.shape[1]
    if C < 128:
        return None
    dy2 = dy.contiguous().view(-1, Cout)
    w2 = w.detach().view(Cout, C)
    if not gemm.hip_mm_ok(dy2, w2):
        return None
    if acc is not None and acc.is_contiguous() and acc.dtype == dy.dtype and acc.numel() == dy2.shape[0] * C:
        gemm.hip_mm(dy2, w2, out=acc.view(-1, C), beta=1.0)
        return acc.view(*dy.shape[:3], C)
    if acc is not None:
        return None
    return gemm.hip_mm(dy2, w2).view(*dy.shape[:3], C)


class GradSink:
    """Hand-off of a residual-branch gradient to the data-gradient GEMM of the convolution that
    consumes the same tensor (ResNet identity blocks): the fused BN + add + ReLU backward parks
    dZ here instead of returning it, and the 1x1 conv's dgrad accumulates into it (beta = 1
    epilogue), so autograd never runs the separate add of the two branch gradients."""
    __slots__ = ('buf', 'armed')

    def __init__(self):
        self.buf = None
        self.armed = False  # set when a convolution's backward has taken the sink


_pending_sink = [None]


class dgrad_sink:
    """Context: the next conv2d_nhwc call adds ``sink.buf`` into its input gradient."""

    def __init__(self, sink):
        self.sink = sink

    def __enter__(self):
        _pending_sink[0] = self.sink
        return self.sink

    def __exit__(self, *exc):
        _pending_sink[0] = None
        return False


class SharedDgrad:
    """Two convolutions reading the same input (a ResNet downsample block's conv1 and shortcut
    conv): the first backward returns its dX and keeps it; the second accumulates its dX into that
    tensor in place (the 1x1 dgrad GEMM's beta = 1 epilogue) and returns None, so autograd runs no
    add of the two branch gradients.  Order-independent; resets for a second backward."""
    __slots__ = ('buf', 'left')

    def __init__(self):
        self.buf = None
        self.left = 2


_shared_by_input = {}


class shared_dgrad:
    """Context: conv2d_nhwc calls on ``x`` (same storage and shape) share ``sh``."""

    def __init__(self, x, sh):
        self.key, self.sh = (x.data_ptr(), tuple(x.shape)), sh

    def __enter__(self):
        _shared_by_input[self.key] = self.sh
        return self.sh

    def __exit__(self, *exc):
        _shared_by_input.pop(self.key, None)
        return False


_stem_enabled = pa_flag('conv_stem')


def stem_ok(x, w, stride, dil):
    """Few-channel forward (the RGB stem) on csrc/conv_stem.hip."""
    Cout, C, R, S = w.shape
    return (_stem_enabled and tuple(dil) == (1, 1) and x.dtype == w.dtype and x.dtype in (torch.bfloat16, torch.float16)
            and N.lib is not None and bool(N.lib.pa_conv_stem_ok(C, -(-Cout // 16) * 16, R, S, stride[0], stride[1])))


def conv2d_fwd_stem(x, w, b, stride, pad, stats=True):
    """y = conv(x, w) for C <= 8: the input rows of RB output rows staged once in LDS, MFMA over
    k = (filter row, s*C + c) with the [Cout][Kp] filter image below; under fused_bn_stats() the
    epilogue also writes the batch-norm slab statistics (one slab per output-row segment).
    C_out % 16 != 0 (ShuffleNet's 3 -> 24 stem): computed over zero filter rows up to the 16-channel
    grain and sliced (no statistics epilogue then)."""
    x = x.contiguous()
    Nb, H, W, C = x.shape
    Cout, _, R, S = w.shape
    if Cout % 16:
        c16 = -(-Cout // 16) * 16
        wp = torch.cat([w, w.new_zeros(c16 - Cout, C, R, S)])
        bp = None if b is None else torch.cat([b, b.new_zeros(c16 - Cout)])
        return conv2d_fwd_stem(x, wp, bp, stride, pad, stats=False)[..., :Cout].contiguous()
    Ho, Wo = _out_hw(H, W, R, S, stride, pad, (1, 1))
    RK, Kp = int(N.lib.pa_conv_stem_rk(C, S)), int(N.lib.pa_conv_stem_kp(C, R, S))
    wimg = torch.zeros(-(-Cout // 64) * 64, Kp, dtype=x.dtype, device=x.device)  # rows past Cout stay zero
    wimg[:Cout, :R * RK].view(Cout, R, RK)[:, :, :S * C] = w.detach().to(x.dtype).permute(0, 2, 3, 1).reshape(Cout, R, S * C)
    y = torch.empty(Nb, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
    bb = b.to(x.dtype).contiguous() if b is not None else None
    rpb = int(N.lib.pa_conv_stem_stat_rows(Wo)) if stats and _want_stats(b) else 0
    parts = None
    if rpb:
        P = Nb * Ho * (-(-Wo // 128))
        parts = torch.empty(2 * P * Cout, dtype=torch.float32, device=x.device)
    N.check(N.lib.pa_conv_stem_fwd(N.ptr(x), N.ptr(wimg), N.ptr(bb), N.ptr(y), N.ptr(parts), Nb, H, W, C, Cout, R, S,
                                   stride[0], stride[1], pad[0], pad[1], Ho, Wo, N.dtcode(x.dtype), N.stream()),
            'conv_stem_fwd')
    if parts is not None:
        _stash_parts(y, parts, P, rpb)
    return y


def _lib_conv_fwd(x, w, b, stride, pad, dil):
    y = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2), w, b, stride, pad, dil)
    return y.permute(0, 2, 3, 1).contiguous()


class _Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil, sink=None, shared=None):
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, dil, b is not None)
        ctx.sink = sink
        ctx.shared = shared
        if _pointwise(w, stride, pad, dil) and w.dtype == torch.bfloat16:
            y = _gemm_fwd_1x1(x, w, b)
            if y is not None:
                return y
        if fwd_ok(w):
            return conv2d_fwd(x, w, b, stride, pad, dil)
        if stem_ok(x, w, stride, dil):
            return conv2d_fwd_stem(x, w, b, stride, pad)
        return _lib_conv_fwd(x, w, b, stride, pad, dil)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, dil, has_b = ctx.cfg
        dy = dy.contiguous()
        gx = gw = gb = None
        pw = _pointwise(w, stride, pad, dil)
        sink = ctx.sink.buf if ctx.sink is not None else None
        if ctx.sink is not None:
            ctx.sink.buf = None
        sh = ctx.shared
        second = sh is not None and sh.buf is not None and ctx.needs_input_grad[0]
        if ctx.needs_input_grad[0] and _bwd_enabled:
            if pw:
                gx = _gemm_dgrad_1x1(dy, w, acc=sh.buf if second else sink)
                if gx is not None:
                    sink = None  # accumulated in the GEMM epilogue
                    if second:
                        gx, second = None, 'done'
            if gx is None and second != 'done':
                gx = conv2d_dgrad_classes(dy, w, x.shape[1:3], stride, pad, dil)
                if gx is None and tuple(stride) == (1, 1) and fwd_ok(w.transpose(0, 1)):
                    # C_out % 32 != 0 (MobileNet pointwise): the stride-1 data gradient as a forward
                    # conv of dY, whose K decomposition pads the channels to 32
                    gx = conv2d_dgrad(dy, w, x.shape[1:3], pad, dil)
        slot_used = False
        if ctx.needs_input_grad[1] and _bwd_enabled and _wgrad_hip and w.shape[0] % 8 == 0:
            C = w.shape[1]
            # the weight's flat-buffer gradient slot: the kernels accumulate into it in place
            # (no AccumulateGrad add), as the Linear weight gradient does (ops/linear.py)
            wp = _param_of(w) if SLOT_ACCUM else None
            slot = flat_grad_slot(wp) if wp is not None else None
            if slot is not None and (slot.dtype != torch.bfloat16 or not slot.is_contiguous()):
                slot = None
            if C % 8:  # RGB stem: zero channels do not change the taps of the real ones
                xp = torch.nn.functional.pad(x, (0, 8 - C % 8))
                gw = conv2d_wgrad(dy, xp, (w.shape[0], xp.shape[3], w.shape[2], w.shape[3]), stride, pad,
                                  dil)[:, :C].contiguous()
            else:
                if pw and w.shape[1] >= 512 and 2 * w.shape[0] >= w.shape[1]:
                    gw = conv2d_wgrad_1x1(dy, x, out=slot)
                    slot_used = gw is not None and slot is not None
                if gw is None:
                    gw = conv2d_wgrad(dy, x, tuple(w.shape), stride, pad, dil, out=slot)
                    slot_used = gw is not None and slot is not None
                    if gw is None:  # transposed 1x1 form: a fresh tensor
                        gw = conv2d_wgrad(dy, x, tuple(w.shape), stride, pad, dil)
            if slot_used:
                notify_grad_ready(wp)
                gw = None
            else:
                gw = gw.to(w.dtype)
        if has_b and ctx.needs_input_grad[2]:
            gb = dy.sum((0, 1, 2), dtype=torch.float32).to(dy.dtype)
        mask = [ctx.needs_input_grad[0] and gx is None and second != 'done',
                ctx.needs_input_grad[1] and gw is None and not slot_used, False]
        if any(mask):  # shapes the hand-written kernels reject: MIOpen NHWC backward
            lx, lw, _ = torch.ops.aten.convolution_backward(
                dy.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2), w, None, list(stride), list(pad), list(dil), False,
                [0, 0], 1, mask)
            if mask[0]:
                gx = lx.permute(0, 2, 3, 1)
            if mask[1]:
                gw = lw
        if sink is not None:  # residual gradient not taken by a GEMM epilogue: plain add
            gx = gx + sink if gx is not None else sink
        if sh is not None and ctx.needs_input_grad[0]:
            if second == 'done':
                pass  # this dX went into the first branch's tensor (GEMM beta = 1)
            elif second:  # this branch's dX came from a non-GEMM kernel: add it to the first's
                sh.buf.add_(gx)
                gx = None
            else:
                sh.buf = gx  # first branch: keep it for the other branch to accumulate into
                # reset at the end of this backward pass whatever happens to the other branch
                # (it may have run on a library conv, or not at all): a retained-graph second
                # backward then starts clean
                torch.autograd.Variable._execution_engine.queue_callback(lambda sh=sh: _reset_shared(sh))
            sh.left -= 1
            if sh.left == 0:
                sh.buf, sh.left = None, 2
        return gx, gw, gb, None, None, None, None, None


def _reset_shared(sh):
    sh.buf, sh.left = None, 2


def conv2d_nhwc(x, w, b, stride, pad, dil):
    sink, _pending_sink[0] = _pending_sink[0], None
    if sink is not None:
        sink.armed = True
    shared = _shared_by_input.get((x.data_ptr(), tuple(x.shape))) if _shared_by_input else None
    return _Conv2dNHWC.apply(x, w, b, tuple(stride), tuple(pad), tuple(dil), sink, shared)


# ---- depthwise convolution (groups == C_in == C_out) on csrc/dwconv.hip
_dw_enabled = pa_flag('hip_dwconv')


def dw_supported(x, w, groups):
    """x: NHWC view; w: [C, 1, R, S] with groups == C (channel multiplier 1), 16-bit dtypes."""
    if not _dw_enabled or x.dim() != 4 or w.dim() != 4 or not x.is_cuda:
        return False
    C = x.shape[3]
    if groups != C or groups == 1 or w.shape[0] != C or w.shape[1] != 1 or C % 8:
        return False
    if x.dtype not in (torch.bfloat16, torch.float16) or w.dtype != x.dtype:
        return False
    return N.lib is not None or N._load() is not None


def _dw_geo(x, w, stride, pad, dil):
    Nb, H, W, C = x.shape
    R, S = w.shape[2], w.shape[3]
    Ho, Wo = _out_hw(H, W, R, S, stride, pad, dil)
    return (Nb, H, W, C, Ho, Wo, R, S, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1])


def _dw_taps(w):
    """[C, 1, R, S] filter -> the tap-major [R*S][C] image the kernels read."""
    C, _, R, S = w.shape
    return w.detach().reshape(C, R * S).t().contiguous()


class _DWConvNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil):
        x = x.contiguous()
        g = _dw_geo(x, w, stride, pad, dil)
        Nb, H, W, C, Ho, Wo = g[:6]
        dt = N.dtcode(x.dtype)
        y = torch.empty(Nb, Ho, Wo, C, dtype=x.dtype, device=x.device)
        bb = b.to(x.dtype).contiguous() if b is not None else None
        N.check(N.lib.pa_dwconv_fwd(N.ptr(x), N.ptr(_dw_taps(w)), N.ptr(bb), N.ptr(y), *g, dt, N.stream()),
                'dwconv_fwd')
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, dil, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, dil, has_b = ctx.cfg
        dy = dy.contiguous()
        g = _dw_geo(x, w, stride, pad, dil)
        Nb, H, W, C, Ho, Wo, R, S = g[:8]
        dt = N.dtcode(x.dtype)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            N.check(N.lib.pa_dwconv_dgrad(N.ptr(dy), N.ptr(_dw_taps(w)), N.ptr(gx), *g, dt, N.stream()),
                    'dwconv_dgrad')
        if ctx.needs_input_grad[1]:
            splits = int(N.lib.pa_dwconv_wgrad_splits(Nb, Ho, Wo, C, R, S))
            ws = torch.empty(splits * R * S * C, dtype=torch.float32, device=x.device)
            gw = torch.empty(C, 1, R, S, dtype=x.dtype, device=x.device)
            N.check(N.lib.pa_dwconv_wgrad(N.ptr(x), N.ptr(dy), N.ptr(ws), N.ptr(gw), *g, splits, 0, dt, N.stream()),
                    'dwconv_wgrad')
            gw = gw.to(w.dtype)
        if has_b and ctx.needs_input_grad[2]:
            gb = dy.sum((0, 1, 2), dtype=torch.float32).to(dy.dtype)
        return gx, gw, gb, None, None, None


def dwconv2d_nhwc(x, w, b, stride, pad, dil):
    """Depthwise conv2d of an NHWC tensor: x [N,H,W,C], w [C,1,R,S] -> y [N,Ho,Wo,C]."""
    if N._load() is None:
        raise RuntimeError("dwconv2d_nhwc: HIP kernel library not loaded: " + str(N.load_error))
    return _DWConvNHWC.apply(x, w, b, tuple(stride), tuple(pad), tuple(dil))


# ---- grouped convolution (1 < groups < C_in, ResNeXt / ShuffleNet-v1) on csrc/gconv.hip
_gc_enabled = pa_flag('hip_gconv')


def _gc_geo(x, w, groups, stride, pad, dil):
    Nb, H, W, C = x.shape
    Cout, _, R, S = w.shape
    Ho, Wo = _out_hw(H, W, R, S, stride, pad, dil)
    return (Nb, H, W, C, Ho, Wo, Cout, groups, R, S, stride[0], stride[1], pad[0], pad[1], dil[0], dil[1])


def gconv_supported(x, w, groups, stride=(1, 1), pad=(0, 0), dil=(1, 1)):
    """x: NHWC view; w: [Cout, C / groups, R, S], 1 < groups < C, C / groups % 4 == 0 and
    Cout / groups % 8 == 0, 16-bit dtypes."""
    if not _gc_enabled or x.dim() != 4 or w.dim() != 4 or not x.is_cuda or groups <= 1:
        return False
    C = x.shape[3]
    if groups >= C or C % groups or w.shape[1] * groups != C or w.shape[0] % groups:
        return False
    if x.dtype not in (torch.bfloat16, torch.float16) or w.dtype != x.dtype:
        return False
    if N.lib is None and N._load() is None:
        return False
    return bool(N.lib.pa_gconv_ok(*_gc_geo(x, w, groups, stride, pad, dil), N.dtcode(x.dtype)))


class _GConvNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, groups, stride, pad, dil):
        x = x.contiguous()
        g = _gc_geo(x, w, groups, stride, pad, dil)
        Nb, H, W, C, Ho, Wo, Cout = g[:7]
        dt = N.dtcode(x.dtype)
        y = torch.empty(Nb, Ho, Wo, Cout, dtype=x.dtype, device=x.device)
        bb = b.to(x.dtype).contiguous() if b is not None else None
        wf = w.detach().permute(2, 3, 1, 0).contiguous()  # [R][S][Cg][Cout]
        N.check(N.lib.pa_gconv_fwd(N.ptr(x), N.ptr(wf), N.ptr(bb), N.ptr(y), *g, dt, N.stream()), 'gconv_fwd')
        ctx.save_for_backward(x, w)
        ctx.cfg = (groups, stride, pad, dil, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        groups, stride, pad, dil, has_b = ctx.cfg
        dy = dy.contiguous()
        g = _gc_geo(x, w, groups, stride, pad, dil)
        Nb, H, W, C, Ho, Wo, Cout, _, R, S = g[:10]
        dt = N.dtcode(x.dtype)
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty_like(x)
            wd = w.detach().permute(2, 3, 0, 1).contiguous()  # [R][S][Cout][Cg]
            N.check(N.lib.pa_gconv_dgrad(N.ptr(dy), N.ptr(wd), N.ptr(gx), *g, dt, N.stream()), 'gconv_dgrad')
        if ctx.needs_input_grad[1]:
            splits = int(N.lib.pa_gconv_wgrad_splits(Nb, Ho, Wo, Cout, groups, R, S, C))
            ws = torch.empty(splits * R * S * Cout * (C // groups), dtype=torch.float32, device=x.device)
            gw = torch.empty(Cout, C // groups, R, S, dtype=x.dtype, device=x.device)
            N.check(N.lib.pa_gconv_wgrad(N.ptr(x), N.ptr(dy), N.ptr(ws), N.ptr(gw), *g, splits, 0, dt, N.stream()),
                    'gconv_wgrad')
            gw = gw.to(w.dtype)
        if has_b and ctx.needs_input_grad[2]:
            gb = dy.sum((0, 1, 2), dtype=torch.float32).to(dy.dtype)
        return gx, gw, gb, None, None, None, None


def gconv2d_nhwc(x, w, b, groups, stride, pad, dil):
    """Grouped conv2d of an NHWC tensor: x [N,H,W,C], w [Cout, C/groups, R, S] -> y [N,Ho,Wo,Cout]."""
    if N._load() is None:
        raise RuntimeError("gconv2d_nhwc: HIP kernel library not loaded: " + str(N.load_error))
    return _GConvNHWC.apply(x, w, b, int(groups), tuple(stride), tuple(pad), tuple(dil))


# ---- transposed convolution (reference gpudnn conv_transpose_kernel.cu) on the same kernels
# conv_transpose2d(x, w) IS the data gradient of conv2d(., w) evaluated at dY = x: the stride-class
# data-gradient kernel computes it; its input gradient is the conv2d forward of dOut with w and its
# filter gradient the conv filter-gradient kernel with the roles of input and output swapped.
def convt_supported(x, w, groups, stride, pad, dil, out_hw):
    """x: NHWC view [N, H, W, Cin]; w: [Cin, Cout, R, S] (paddle's transposed-conv layout)."""
    if not (_enabled and _bwd_enabled) or groups != 1 or x.dim() != 4 or w.dim() != 4 or not x.is_cuda:
        return False
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.shape[3] != w.shape[0]:
        return False
    if N.lib is None and N._load() is None:
        return False
    Cin, Cout, R, S = w.shape
    if not bool(N.lib.pa_conv2d_fwd_ok(Cout, Cin, R, S)) or not bool(N.lib.pa_conv2d_wgrad_ok(Cout, Cin)):
        return False
    ok = _dgrad_plan((Cin, Cout, R, S), tuple(out_hw), tuple(stride), tuple(pad), tuple(dil), x.device)[0]
    return bool(ok)


class _ConvT2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, dil, out_hw):
        x = x.contiguous()
        y = conv2d_dgrad_classes(x, w, out_hw, stride, pad, dil)
        if y is None:
            raise RuntimeError("conv_transpose2d: geometry rejected by the data-gradient kernel")
        if b is not None:
            y = y + b.to(y.dtype)
        ctx.save_for_backward(x, w)
        ctx.cfg = (stride, pad, dil, b is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, dil, has_b = ctx.cfg
        dy = dy.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:  # conv2d forward of dOut with the same filter
            gx = conv2d_fwd(dy, w, None, stride, pad, dil)
        if ctx.needs_input_grad[1]:  # filter gradient of that conv: its input is dOut, its dY is x
            gw = conv2d_wgrad(x, dy, tuple(w.shape), stride, pad, dil).to(w.dtype)
        if has_b and ctx.needs_input_grad[2]:
            gb = dy.sum((0, 1, 2), dtype=torch.float32).to(dy.dtype)
        return gx, gw, gb, None, None, None, None


def conv_transpose2d_nhwc(x, w, b, stride, pad, dil, out_hw):
    """Transposed conv2d of an NHWC tensor: x [N,H,W,Cin], w [Cin,Cout,R,S] -> [N,Ho,Wo,Cout]."""
    return _ConvT2dNHWC.apply(x, w, b, tuple(stride), tuple(pad), tuple(dil), tuple(out_hw))
