"""GEMM entry points.

bf16 GEMMs of the training step (Linear forward / dgrad / weight gradient, the tied LM head)
run on the hand-written 8-phase ping-pong MFMA kernel (csrc/gemm8.hip via ``hip_mm``); shapes
outside its contract (K % 64, odd leading dims, fp32/fp16) go to the library through torch.
FP8 (OCP e4m3fn / e5m2, CDNA4 — NOT the MI300 fnuz encoding) runs on the hand-written
block-scaled MFMA kernel (``hip_fp8_mm``, 2x the bf16 MFMA rate) with per-tensor scales;
``torch._scaled_mm`` only for layouts that kernel does not take.

Reference: paddle/phi/kernels/funcs/blas/blaslt_impl.cu.h, fusion/fp8_gemm.
"""
from ..framework.flags import pa_flag  # noqa: E402
import os

import torch

from . import _native as N
from .workspace import workspace as _new_workspace

_GEMM_WS = _new_workspace('gemm_partials')


def _op_layout(t):
    """(trans, ld) of a 2-D bf16 operand: 0 = row-major [rows][cols], 1 = a transposed view."""
    if t.stride(1) == 1 and t.stride(0) >= t.shape[1]:
        return 0, t.stride(0)
    if t.stride(0) == 1 and t.stride(1) >= t.shape[0]:
        return 1, t.stride(1)
    return None, None


def _workspace(n, device):
    """fp32 split-K / skinny-GEMM partials (capture-safe, ops/workspace.py)."""
    return _GEMM_WS.get(n, torch.float32, device, min_numel=1 << 20)


def hip_mm_ok(a, b, splitk=1):
    if a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or a.dim() != 2 or b.dim() != 2:
        return False
    ta, lda = _op_layout(a)
    tb, ldb = _op_layout(b)
    if ta is None or tb is None or a.shape[1] != b.shape[0]:
        return False
    if a.data_ptr() % 16 or b.data_ptr() % 16:
        return False
    M, K = a.shape
    N_ = b.shape[1]
    return N.lib is not None and bool(N.lib.pa_gemm_ok(M, N_, K, lda, ldb, N_, splitk))


def hip_mm(a, b, out=None, bias=None, alpha=1.0, beta=0.0, splitk=1):
    """out[M,N] = alpha * a @ b (+ beta * out) (+ bias) on the hand-written MFMA GEMM (csrc/gemm.hip).

    a: [M,K] bf16, row-major or a transposed view of a [K,M] tensor; b: [K,N] bf16, row-major
    or a transposed view of [N,K].  ``out`` (row-major, unit column stride) is written in
    place (with beta = 1 this is the in-place weight-gradient accumulate).
    """
    ta, lda = _op_layout(a)
    # B's "trans" flag in the kernel means stored [N][K] (k contiguous)
    tb, ldb = _op_layout(b)
    M, K = a.shape
    N_ = b.shape[1]
    if out is None:
        out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
        beta = 0.0
    assert out.stride(1) == 1 and out.shape == (M, N_)
    ws = _workspace(splitk * M * N_, a.device) if splitk > 1 else None
    N.check(N.lib.pa_gemm_bf16(N.ptr(a), N.ptr(b), N.ptr(out), N.ptr(bias), N.ptr(ws), M, N_, K, lda, ldb,
                               out.stride(0), ta, tb, float(alpha), float(beta), splitk, N.stream()), 'gemm_bf16')
    return out


_hip_gemm = pa_flag('hip_gemm')


def epi_ok(a, b, out_cols):
    """Shape/layout contract of the fused-epilogue GEMMs (mm_epi): a k-contiguous [M,K]."""
    if not _hip_gemm or not a.is_cuda or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        return False
    ta, lda = _op_layout(a)
    tb, ldb = _op_layout(b)
    if ta != 0 or tb is None or a.data_ptr() % 16 or b.data_ptr() % 16 or N._load() is None:
        return False
    return bool(N.lib.pa_gemm8_ok(a.shape[0], out_cols, a.shape[1], lda, ldb, out_cols, 0, tb, 1))


def mm_epi(a, b, epi, aux, bias=None, out=None, colsum_part=None):
    """Fused-epilogue GEMM of the MLP (csrc/gemm8.hip pa_gemm8_bf16_epi, schedule 11).

    epi 2 (fc1 forward): h = a @ b + bias; returns gelu_tanh(h) and writes gelu_tanh'(h) to ``aux``;
    epi 3 (fc2 dgrad):   returns (a @ b) * aux.   a: [M,K] row-major; b: [K,N]
    (row-major or a transposed view of [N,K]); aux: bf16 [M,N] contiguous.
    colsum_part (epi 3 only): fp32 [ceil(M/128) * N] receiving per-128-row-slab column sums of the
    result (the fc1 bias gradient, finished by fused.colsum_finish_parts)."""
    tb, ldb = _op_layout(b)
    M, K = a.shape
    N_ = b.shape[1]
    if out is None:
        out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
    assert aux.shape == (M, N_) and aux.is_contiguous() and out.is_contiguous()
    if colsum_part is not None:
        assert epi == 3 and colsum_part.dtype == torch.float32 and colsum_part.numel() >= -(-M // 128) * N_
        epi, bias = 4, colsum_part
    N.check(N.lib.pa_gemm8_bf16_epi(N.ptr(a), N.ptr(b), N.ptr(out), N.ptr(bias), N.ptr(aux), M, N_, K, a.stride(0),
                                    ldb, N_, tb, 1.0, int(epi), N.stream()), f'gemm_epi{epi}')
    return out


_ACT_EPI = {'relu': 6, 'gelu': 7, 'gelu_tanh': 8}


def mm_act(a, b, bias, act):
    """act(a @ b + bias) with the bias and the activation (relu / gelu erf / gelu tanh) in the
    GEMM's wave-staged epilogue (csrc/gemm8.hip pa_gemm8_bf16_act) — the inference fc_fuse_pass
    form: no derivative output, no separate activation pass.  a: [M, K] k-contiguous bf16; b: [K, N]
    (row-major or a transposed view of [N, K]); contract: ``epi_ok(a, b, N)``."""
    tb, ldb = _op_layout(b)
    M, K = a.shape
    N_ = b.shape[1]
    out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
    bb = None if bias is None else bias.to(torch.bfloat16).contiguous()
    N.check(N.lib.pa_gemm8_bf16_act(N.ptr(a), N.ptr(b), N.ptr(out), N.ptr(bb), M, N_, K, a.stride(0), ldb, N_, tb,
                                    1.0, _ACT_EPI[act], N.stream()), f'gemm_act_{act}')
    return out


def mm_bn_stats(a, b):
    """out = a @ b on the fused-epilogue GEMM (epi 5) plus the batch-norm column statistics of
    every 128-row slab of out: returns (out, parts fp32 [2][P][N] (slab means, then M2s), P)."""
    tb, ldb = _op_layout(b)
    M, K = a.shape
    N_ = b.shape[1]
    out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
    P = -(-M // 128)
    parts = torch.empty(2 * P * N_, dtype=torch.float32, device=a.device)
    N.check(N.lib.pa_gemm8_bf16_epi(N.ptr(a), N.ptr(b), N.ptr(out), None, N.ptr(parts), M, N_, K, a.stride(0),
                                    ldb, N_, tb, 1.0, 5, N.stream()), 'gemm_epi5')
    return out, parts, P


def _splitk_for(M, N_, K):
    """Split-K factor for outputs with too few 256x256 tiles to fill 256 CUs: the split (2..32 slices
    of >= 2048 k each, the last one possibly shorter but at least half a slice) that puts the most
    blocks within one round of the chip.  Weight gradients
    over many tokens: GPT-3 out-projection 2048x2048 64 tiles -> 4 (1058 TF), ERNIE-base at 32768
    tokens 768x2304 27 tiles -> 8 (193 -> 126 us), 768x768 9 tiles -> 16 (183 -> 66 us), 768x3072
    36 tiles -> 4 (profiles/r5bb_wgrad_splitk_ab.log)."""
    tiles = -(-M // 256) * -(-N_ // 256)
    if tiles >= 128 or K % 64:
        return 1
    kb = K // 64
    best, best_blocks = 1, tiles
    for s in range(2, 33):
        q = -(-kb // s)  # k-blocks per slice (the last slice may be shorter)
        if q * 64 < 2048 or tiles * s > 256 or kb - (s - 1) * q < max(2, q // 2):
            continue
        if tiles * s > best_blocks:
            best, best_blocks = s, tiles * s
    return best


_skinny = pa_flag('skinny_gemm')


def skinny_ok(a, b):
    """Decode-shaped GEMM contract (csrc/skinny_gemm.hip): a [M<=64, K] k-contiguous, b [K, N]
    row-major or a transposed view of [N, K]."""
    if not (_skinny and a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2
            and b.dim() == 2 and a.stride(1) == 1 and a.shape[1] == b.shape[0]):
        return False
    if b.stride(1) == 1:
        ldw = b.stride(0)
    elif b.stride(0) == 1:
        ldw = b.stride(1)
    else:
        return False
    if a.data_ptr() % 16 or b.data_ptr() % 16 or N._load() is None:
        return False
    return bool(N.lib.pa_skinny_ok(a.shape[0], b.shape[1], a.shape[1], a.stride(0), ldw))


def skinny_mm(a, b, bias=None, out=None):
    """out[M, N] = a @ b (+ bias) for M <= 64 (decode steps) on the weight-streaming MFMA kernel:
    in-register 8x8 transposes of n-major weight blocks feed v_mfma_f32_16x16x32_bf16 directly,
    K split over ~2 blocks per CU with an fp32 partial sum (csrc/skinny_gemm.hip)."""
    M, K = a.shape
    N_ = b.shape[1]
    kmaj = b.stride(1) != 1
    ldw = b.stride(1) if kmaj else b.stride(0)
    if out is None:
        out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
    assert out.stride(1) == 1 and out.stride(0) % 8 == 0
    bb = bias.to(torch.bfloat16).contiguous() if bias is not None else None
    ws = _workspace(int(N.lib.pa_skinny_ws_floats(M, N_, K)), a.device)
    N.check(N.lib.pa_skinny_gemm(N.ptr(a), N.ptr(b), N.ptr(bb), N.ptr(out), N.ptr(ws), M, N_, K, a.stride(0), ldw,
                                 out.stride(0), int(kmaj), N.stream()), 'skinny_gemm')
    return out


def _skinny_wins(M, N_, K):
    """Where the skinny kernel beats the library (profiles/r3s3_decode_gemm.log, Llama-2-13B layer
    shapes): every shape at M <= 16 (out 22.9 -> 16.8 us, ffn2 53.3 -> 26.1, ffn1 59 -> 48, qkv
    even); at 16 < M <= 64 only the deep-K shapes (ffn2: 60 -> 33 us at M 32, 75 -> 46 at M 64)."""
    return _skinny and (M <= 16 or (M <= 64 and K >= 2 * N_))


def _round_split(a, b, out, beta=0.0):
    """Few-round GEMMs whose last round of 256x256 tiles leaves most CUs idle (the tied LM-head
    weight gradient: 197 x 8 = 1576 tiles = 6 full rounds + 40 tiles): the rows of the full rounds
    run as one GEMM and the remaining tile rows as a split-K GEMM (4x the work items at 1/4 the
    depth), so the tail costs about a quarter round instead of a whole one.  beta (accumulate
    into ``out``) is honoured by both parts.  None when it does not apply."""
    M, K = a.shape
    N_ = b.shape[1]
    tm, tn = -(-M // 256), -(-N_ // 256)
    tiles = tm * tn
    full = tiles // 256
    tail = tiles - full * 256
    if full == 0 or full > 12 or tail == 0 or tail * 10 > 256 * 3:
        return None  # many rounds (the tail is a small share) or a well-filled last round
    m1 = (full * 256 // tn) * 256  # rows covered by whole tile rows inside the full rounds
    if m1 <= 0 or m1 >= M:
        return None
    rest_tiles = -(-(M - m1) // 256) * tn
    sk = 1
    for s_ in (8, 4, 2):
        if rest_tiles * s_ <= 256 and K % (64 * s_) == 0 and K // s_ >= 512:
            sk = s_
            break
    if sk == 1:
        return None
    a1, a2 = a[:m1], a[m1:]
    if not (hip_mm_ok(a1, b, 1) and hip_mm_ok(a2, b, sk)):
        return None
    if out is None:
        out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
        beta = 0.0
    hip_mm(a1, b, out=out[:m1], beta=beta)
    hip_mm(a2, b, out=out[m1:], beta=beta, splitk=sk)  # beta applied by the split-K reduce
    return out


def mm(a, b, out=None, bias=None, beta=0.0):
    """out = a @ b (+ beta*out) (+ bias) on the hand-written kernels when the operands fit their
    contract (M <= 64: the decode-shaped skinny GEMM; else the 8-phase MFMA GEMM), else on the
    library (torch).  a: [M,K], b: [K,N] (either may be a transposed view)."""
    if a.is_cuda and b.dim() == 2 and b.shape[1] < 8 and out is None and beta == 0.0:
        r = _tiny_n(a, b, bias)
        if r is not None:
            return r
    if a.is_cuda and _skinny_wins(a.shape[0], b.shape[1], a.shape[1]) and beta == 0.0 and skinny_ok(a, b) and (
            out is None or (
            out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.stride(0) % 8 == 0)):
        return skinny_mm(a, b, bias=bias, out=out)
    if _hip_gemm and a.is_cuda and hip_mm_ok(a, b, 1) and (bias is None or (
            bias.dtype == torch.bfloat16 and bias.is_contiguous())) and (out is None or (
            out.dtype == torch.bfloat16 and out.stride(1) == 1)):
        sk = _splitk_for(a.shape[0], b.shape[1], a.shape[1]) if bias is None else 1
        if sk > 1 and not hip_mm_ok(a, b, sk):
            sk = 1
        if sk == 1 and bias is None:
            r = _round_split(a, b, out, beta if out is not None else 0.0)
            if r is not None:
                return r
        return hip_mm(a, b, out=out, bias=bias, beta=beta if out is not None else 0.0, splitk=sk)
    if out is None:
        return torch.addmm(bias, a, b) if bias is not None else torch.mm(a, b)
    if beta == 0.0:
        torch.mm(a, b, out=out)
    else:
        out.addmm_(a, b, beta=beta)
    if bias is not None:
        out.add_(bias)
    return out


def _tiny_n(a, b, bias):
    """A GEMM with fewer than 8 output columns (a classifier head: [M, K] @ [K, 2]) as its transpose
    y^T = b^T @ a^T on the decode-shaped skinny kernel: b^T's < 8 rows are its short side (padded to
    8 with zero rows), the M activation rows its N.  None when the operands do not fit."""
    M, K = a.shape
    n = b.shape[1]
    if not _skinny or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 or M % 8 or M < 8 or a.stride(1) != 1:
        return None
    wt = torch.zeros(8, K, dtype=torch.bfloat16, device=a.device)
    wt[:n].copy_(b.t())
    at = a.t()  # [K, M]: a transposed view of the k-contiguous [M, K]
    if not skinny_ok(wt, at):
        return None
    yt = skinny_mm(wt, at)  # [8, M]
    y = yt[:n].t()
    if bias is not None:
        y = y + bias.to(y.dtype)
    return y.contiguous()


def wgrad_accumulate(x2, dy2, gw):
    """gw[in, out] += x2^T @ dy2 (x2: [tokens, in], dy2: [tokens, out]) — the weight-gradient GEMM
    on the hand-written kernel (both operands m/n-contiguous: k-half staged images read with
    ds_read_b64_tr_b16, beta = 1 epilogue accumulating in place; split-K for small outputs).
    Returns False when the caller should use the library."""
    if not _hip_gemm or gw.dtype != torch.bfloat16 or not gw.is_contiguous() or not hip_mm_ok(x2.t(), dy2, 1):
        return False
    mm(x2.t(), dy2, out=gw, beta=1.0)
    return True


def wgrad_tiles(gw):
    """256x256 output tiles of a weight gradient."""
    return -(-gw.shape[0] // 256) * -(-gw.shape[1] // 256)


def wgrad_grouped_ok(x2, dy2, gw):
    return (_hip_gemm and x2.is_cuda and gw.dtype == torch.bfloat16 and gw.is_contiguous() and
            hip_mm_ok(x2.t(), dy2, 1) and _op_layout(x2.t())[0] == 1 and _op_layout(dy2)[0] == 0)


def wgrad_accumulate_grouped2(a, b):
    """Two weight gradients gw += x^T @ dy (a, b: (x2, dy2, gw), the same token count) in ONE
    launch of the weight-gradient GEMM (csrc/gemm8.hip pa_gemm8_wgrad_grouped2): their tiles fill
    one round of the chip together where each alone would leave CUs idle or need split-K."""
    (xa, da, ga), (xb, db, gb) = a, b
    K = xa.shape[0]
    assert xb.shape[0] == K and da.shape[0] == K and db.shape[0] == K
    at, bt = xa.t(), xb.t()
    N.check(N.lib.pa_gemm8_wgrad_grouped2(
        N.ptr(at), N.ptr(da), N.ptr(ga), ga.shape[0], ga.shape[1], _op_layout(at)[1], _op_layout(da)[1], ga.stride(0),
        N.ptr(bt), N.ptr(db), N.ptr(gb), gb.shape[0], gb.shape[1], _op_layout(bt)[1], _op_layout(db)[1],
        gb.stride(0), K, 1.0, 1.0, N.stream()), 'gemm_wgrad_grouped2')


def transpose2d(x):
    """x^T materialised (csrc/act.hip ``pa_transpose2d``: 64x64 LDS tiles, 16-byte loads/stores)."""
    R, C = x.shape
    if N._load() is None:
        raise RuntimeError("transpose2d: HIP kernel library not loaded: " + str(N.load_error))
    y = torch.empty((C, R), dtype=x.dtype, device=x.device)
    N.check(N.lib.pa_transpose2d(N.ptr(x), N.ptr(y), R, C, x.element_size(), N.stream()), 'transpose2d')
    return y


_kmajor_fwd = pa_flag('kmajor_fwd')


def kmajor_weight(x2, w):
    """K-major copy W^T ([out, in]) of a paddle [in, out] weight for the forward GEMM, or None.

    Both operands K-major is the hand-written GEMM's fastest layout (an LDS-staged N-major B tile
    needs a transposing read); the transpose of a 2048x8192 weight costs ~15 us, so the copy pays
    off once the token count is large (training micro-batches): GPT-3 1.3B step (16384 rows)
    129.1-129.5 ms with the copies vs 130.2-130.5 ms reading W directly
    (profiles/r3s3_kmajor_fwd_ab.log; round 1's hipBLASLt measurement: profiles/fwd_layout_r1.log),
    while the Llama-2 13B layer stack (8192 rows, 5120 x 27648 weights) runs 0.7 ms faster without
    them (profiles/r6w_llama_kmajor_ab.log): the copy costs in proportion to the weight, the gain in
    proportion to the rows, so it is made from 12288 rows on.
    """
    if not _kmajor_fwd or x2.shape[0] < 12288 or w.dtype not in (torch.bfloat16, torch.float16):
        return None
    if w.dim() != 2 or not w.is_contiguous() or w.shape[0] % 64 or w.shape[1] % 64 or not x2.is_cuda:
        return None
    if N._load() is None:
        return None
    return transpose2d(w)


_FP8_FMT = {torch.float8_e4m3fn: 0, torch.float8_e5m2: 1}
# fp8 GEMM schedule: the 8-phase kernel (csrc/gemm8x.hip pa_gemm8_fp8, default) or the round-1
# two-stage kernel (csrc/gemm.hip pa_gemm_fp8; PADDLE_AMD_FP8_8PHASE=0, A/B only)
_fp8_8phase = pa_flag('fp8_8phase')


_FP8_WS = _new_workspace('fp8_splitk')


def _fp8_splitk(M, N_, K):
    """Split-K factor of an fp8 GEMM whose 256x256 output tiles cannot fill the chip (the fp8 Linear
    weight gradient: in x out features over a token-count K): the split (slices of >= 1024 k, the
    last one possibly shorter) that puts the most blocks within one round of the chip (768x3072
    over 32768 tokens: one round at s = 4 beat 1.1 rounds at s = 8, 112 vs 127 us,
    profiles/r5ss_fp8_wgrad_splitk_ab.log; uneven s = 7 fills 252 CUs)."""
    tiles = -(-M // 256) * -(-N_ // 256)
    if tiles >= 128 or K % 128:
        return 1
    kb = K // 128  # 128-value k-tiles
    best, best_blocks = 1, tiles
    for s in range(2, 33):
        q = -(-kb // s)  # k-tiles per slice (the last slice may be shorter, but at least half a slice)
        if q * 128 < 1024 or tiles * s > FP8_SPLITK_MAX_BLOCKS[0] or kb - (s - 1) * q < max(2, q // 2):
            continue
        if tiles * s > best_blocks:
            best, best_blocks = s, tiles * s
    return best


FP8_SPLITK_MAX_BLOCKS = [256]  # block budget of the fp8 split-K rule (tools/fp8_wgrad_splitk_ab.py)


def hip_fp8_ok(a, w):
    """a: [M,K] fp8 row-major; w: [N,K] fp8 row-major (the weight of an fp8 Linear)."""
    if a.dtype not in _FP8_FMT or w.dtype not in _FP8_FMT or a.dim() != 2 or w.dim() != 2:
        return False
    if a.stride(1) != 1 or w.stride(1) != 1 or a.shape[1] != w.shape[1] or a.data_ptr() % 16 or w.data_ptr() % 16:
        return False
    if N.lib is None and N._load() is None:
        return False
    return bool(N.lib.pa_gemm_fp8_ok(a.shape[0], w.shape[0], a.shape[1], a.stride(0), w.stride(0), w.shape[0]))


def hip_fp8_mm(a, w, scale_a=None, scale_b=None, bias=None, out=None, alpha=1.0, beta=0.0):
    """out[M,N] (bf16) = alpha * scale_a * scale_b * a @ w^T (+ beta*out) (+ bias) on the
    hand-written CDNA4 fp8 kernel (v_mfma_scale_f32_16x16x128_f8f6f4 on the 8-phase ping-pong
    schedule, csrc/gemm8x.hip; the older two-stage kernel of csrc/gemm.hip for A/B).
    scale_a / scale_b: device fp32 scalars (dequant scales), read on the GPU (no host sync)."""
    M, K = a.shape
    N_ = w.shape[0]
    if out is None:
        out = torch.empty(M, N_, dtype=torch.bfloat16, device=a.device)
        beta = 0.0
    assert out.dtype == torch.bfloat16 and out.stride(1) == 1 and out.shape == (M, N_)
    sa = scale_a.float().reshape(1) if scale_a is not None else None
    sb = scale_b.float().reshape(1) if scale_b is not None else None
    sk = _fp8_splitk(M, N_, K)
    if _fp8_8phase and sk > 1 and N.lib.pa_gemm8_fp8_ok(M, N_, K, a.stride(0), w.stride(0), out.stride(0)):
        # few output tiles over a deep K (the fp8 weight gradient): K split over the grid, fp32 slabs
        ws = _FP8_WS.get(sk * M * N_, torch.float32, a.device)
        N.check(N.lib.pa_gemm8_fp8_splitk(N.ptr(a), N.ptr(w), N.ptr(out), N.ptr(bias), N.ptr(sa), N.ptr(sb), N.ptr(ws),
                                          M, N_, K, a.stride(0), w.stride(0), out.stride(0), float(alpha),
                                          float(beta), _FP8_FMT[a.dtype], _FP8_FMT[w.dtype], sk, N.stream()),
                'gemm8_fp8_splitk')
        return out
    if _fp8_8phase and N.lib.pa_gemm8_fp8_ok(M, N_, K, a.stride(0), w.stride(0), out.stride(0)):
        # the 8-phase ping-pong schedule of the bf16 GEMM with one scaled fp8 MFMA per 128-byte k-tile
        N.check(N.lib.pa_gemm8_fp8(N.ptr(a), N.ptr(w), N.ptr(out), N.ptr(bias), N.ptr(sa), N.ptr(sb), M, N_, K,
                                   a.stride(0), w.stride(0), out.stride(0), float(alpha), float(beta),
                                   _FP8_FMT[a.dtype], _FP8_FMT[w.dtype], N.stream()), 'gemm8_fp8')
        return out
    N.check(N.lib.pa_gemm_fp8(N.ptr(a), N.ptr(w), N.ptr(out), N.ptr(bias), N.ptr(sa), N.ptr(sb), M, N_, K, a.stride(0),
                              w.stride(0), out.stride(0), float(alpha), float(beta), _FP8_FMT[a.dtype],
                              _FP8_FMT[w.dtype], N.stream()), 'gemm_fp8')
    return out


def fp8_quantize(x, dtype=torch.float8_e4m3fn):
    amax = x.detach().abs().amax().float().clamp_min(1e-12)
    fmax = torch.finfo(dtype).max
    scale = (fmax / amax).reciprocal()
    return (x.float() / scale).clamp(-fmax, fmax).to(dtype), scale


def fp8_gemm(x, y, transpose_x=False, transpose_y=False, bias=None, scale=1.0, output_dtype='bfloat16',
             activation_type='identity'):
    from ..core.tensor import _wrap, _unwrap
    a, b = _unwrap(x), _unwrap(y)
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    od = {'bfloat16': torch.bfloat16, 'float16': torch.float16, 'float32': torch.float32}.get(str(output_dtype).replace('paddle.', ''),
                                                                                               torch.bfloat16)
    if a.dtype not in (torch.float8_e4m3fn, torch.float8_e5m2):
        a, sa = fp8_quantize(a)
    else:
        sa = torch.tensor(1.0, device=a.device)
    if b.dtype not in (torch.float8_e4m3fn, torch.float8_e5m2):
        b, sb = fp8_quantize(b)
    else:
        sb = torch.tensor(1.0, device=b.device)
    a2 = a.reshape(-1, a.shape[-1]) if a.dim() > 2 else a
    wt = b.t() if b.dim() == 2 else None  # [N, K]
    if (a2.is_cuda and wt is not None and od == torch.bfloat16 and hip_fp8_ok(a2.contiguous(), wt.contiguous())):
        bb = _unwrap(bias) if bias is not None else None
        if bb is not None and (bb.dtype != torch.bfloat16 or not bb.is_contiguous()):
            bb = bb.to(torch.bfloat16).contiguous()
        out = hip_fp8_mm(a2.contiguous(), wt.contiguous(), scale_a=sa, scale_b=sb, bias=bb, alpha=scale)
        out = out.reshape(*a.shape[:-1], out.shape[-1])
    else:
        try:
            out = torch._scaled_mm(a.contiguous(), b.t().contiguous().t(), scale_a=sa.float(), scale_b=sb.float(),
                                   out_dtype=od)
        except Exception:  # CPU / unsupported shape: exact dequantised matmul
            out = (a.float() * sa) @ (b.float() * sb)
            out = out.to(od)
        out = out * scale if scale != 1.0 else out
        if bias is not None:
            out = out + _unwrap(bias).to(out.dtype)
    if activation_type == 'gelu':
        out = torch.nn.functional.gelu(out)
    elif activation_type == 'relu':
        out = torch.relu(out)
    return _wrap(out)
