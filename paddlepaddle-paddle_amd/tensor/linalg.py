"""paddle linalg API (reference: python/paddle/tensor/linalg.py, python/paddle/linalg.py).

``matmul`` / ``mm`` / ``bmm`` / two-operand ``einsum`` are the dense GEMM entry points: bf16 / fp16
operands on the GPU run the hand-written MFMA GEMM (ops/matmul.py: batched with broadcasting,
transposes read in place); other dtypes / devices / shapes outside the kernel contract use torch.
"""
import torch

from ._helpers import _w, _u, _axis, Tensor
from ..core.amp_dispatch import amp_op as _amp_op
from ..ops import matmul as _hm


@_amp_op('matmul_v2')
def matmul(x, y, transpose_x=False, transpose_y=False, name=None):
    a, b = _u(x), _u(y)
    if transpose_x:
        a = a.transpose(-1, -2) if a.dim() > 1 else a
    if transpose_y:
        b = b.transpose(-1, -2) if b.dim() > 1 else b
    return _w(_hm.matmul(a, b))


@_amp_op('matmul_v2')
def mm(input, mat2, name=None):  # noqa: A002
    return _w(_hm.matmul(_u(input), _u(mat2)))


@_amp_op('matmul_v2')
def bmm(x, y, name=None):
    a, b = _u(x), _u(y)
    if a.dim() != 3 or b.dim() != 3 or a.shape[0] != b.shape[0]:
        return _w(torch.bmm(a, b))  # torch's error for mismatched shapes
    return _w(_hm.matmul(a, b))


def dot(x, y, name=None):
    a, b = _u(x), _u(y)
    if a.dim() == 1:
        return _w(torch.dot(a, b))
    return _w((a * b).sum(-1))


def mv(x, vec, name=None):
    return _w(torch.mv(_u(x), _u(vec)))


@_amp_op('einsum')
def einsum(equation, *operands):
    if len(operands) == 1 and isinstance(operands[0], (list, tuple)):
        operands = operands[0]
    return _w(_hm.einsum(equation, *[_u(o) for o in operands]))


@_amp_op('pnorm')
def norm(x, p=None, axis=None, keepdim=False, name=None):
    t = _u(x)
    a = _axis(axis)
    if p is None:
        p = 'fro'
    if p == 'fro':
        if a is None:
            return _w(torch.linalg.vector_norm(t, 2, keepdim=keepdim))
        if isinstance(a, int):
            return _w(torch.linalg.vector_norm(t, 2, dim=a, keepdim=keepdim))
        return _w(torch.linalg.matrix_norm(t, 'fro', dim=a, keepdim=keepdim))
    if p == 'nuc':
        return _w(torch.linalg.matrix_norm(t, 'nuc', dim=a if a is not None else (-2, -1), keepdim=keepdim))
    p = float(p)
    if a is None:
        return _w(torch.linalg.vector_norm(t.flatten(), p, keepdim=False).reshape([1] * t.dim() if keepdim else []))
    if isinstance(a, tuple) and len(a) == 2 and p not in (float('inf'), float('-inf')) and False:
        return _w(torch.linalg.matrix_norm(t, p, dim=a, keepdim=keepdim))
    return _w(torch.linalg.vector_norm(t, p, dim=a, keepdim=keepdim))


def vector_norm(x, p=2.0, axis=None, keepdim=False, name=None):
    return _w(torch.linalg.vector_norm(_u(x), p, dim=_axis(axis), keepdim=keepdim))


def matrix_norm(x, p='fro', axis=[-2, -1], keepdim=False, name=None):  # noqa: B006
    return _w(torch.linalg.matrix_norm(_u(x), p, dim=tuple(axis), keepdim=keepdim))


def cond(x, p=None, name=None):
    return _w(torch.linalg.cond(_u(x), p))


def det(x, name=None):
    return _w(torch.linalg.det(_u(x)))


def slogdet(x, name=None):
    s, l = torch.linalg.slogdet(_u(x))
    return _w(torch.stack([s, l]))


def inv(x, name=None):
    return _w(torch.linalg.inv(_u(x)))


def pinv(x, rcond=1e-15, hermitian=False, name=None):
    return _w(torch.linalg.pinv(_u(x), rtol=rcond, hermitian=hermitian))


def solve(x, y, left=True, name=None):
    return _w(torch.linalg.solve(_u(x), _u(y), left=left))


def triangular_solve(x, y, upper=True, transpose=False, unitriangular=False, name=None):
    a = _u(x)
    if transpose:
        a = a.transpose(-1, -2)
        upper = not upper
    return _w(torch.linalg.solve_triangular(a, _u(y), upper=upper, unitriangular=unitriangular))


def cholesky(x, upper=False, name=None):
    return _w(torch.linalg.cholesky(_u(x), upper=upper))


def cholesky_solve(x, y, upper=False, name=None):
    return _w(torch.cholesky_solve(_u(x), _u(y), upper=upper))


def cholesky_inverse(x, upper=False, name=None):
    return _w(torch.cholesky_inverse(_u(x), upper=upper))


def qr(x, mode='reduced', name=None):
    q, r = torch.linalg.qr(_u(x), mode=mode)
    return _w(r) if mode == 'r' else (_w(q), _w(r))


def svd(x, full_matrices=False, name=None):
    u, s, vh = torch.linalg.svd(_u(x), full_matrices=full_matrices)
    return _w(u), _w(s), _w(vh)


def svd_lowrank(x, q=None, niter=2, M=None, name=None):
    u, s, v = torch.svd_lowrank(_u(x), q=q, niter=niter, M=_u(M))
    return _w(u), _w(s), _w(v)


def pca_lowrank(x, q=None, center=True, niter=2, name=None):
    u, s, v = torch.pca_lowrank(_u(x), q=q, center=center, niter=niter)
    return _w(u), _w(s), _w(v)


def svdvals(x, name=None):
    return _w(torch.linalg.svdvals(_u(x)))


def eig(x, name=None):
    w, v = torch.linalg.eig(_u(x))
    return _w(w), _w(v)


def eigvals(x, name=None):
    return _w(torch.linalg.eigvals(_u(x)))


def eigh(x, UPLO='L', name=None):
    w, v = torch.linalg.eigh(_u(x), UPLO=UPLO)
    return _w(w), _w(v)


def eigvalsh(x, UPLO='L', name=None):
    return _w(torch.linalg.eigvalsh(_u(x), UPLO=UPLO))


def lstsq(x, y, rcond=None, driver=None, name=None):
    r = torch.linalg.lstsq(_u(x), _u(y), rcond=rcond, driver=driver)
    return _w(r.solution), _w(r.residuals), _w(r.rank), _w(r.singular_values)


def lu(x, pivot=True, get_infos=False, name=None):
    lu_, piv, info = torch.linalg.lu_factor_ex(_u(x), pivot=pivot)
    piv = piv.to(torch.int32)
    return (_w(lu_), _w(piv), _w(info)) if get_infos else (_w(lu_), _w(piv))


def lu_unpack(x, y, unpack_ludata=True, unpack_pivots=True, name=None):
    p, l, u = torch.lu_unpack(_u(x), _u(y), unpack_ludata, unpack_pivots)
    return _w(p), _w(l), _w(u)


def matrix_power(x, n, name=None):
    return _w(torch.linalg.matrix_power(_u(x), n))


def matrix_rank(x, tol=None, hermitian=False, atol=None, rtol=None, name=None):
    return _w(torch.linalg.matrix_rank(_u(x), atol=atol if tol is None else tol, rtol=rtol, hermitian=hermitian))


def matrix_exp(x, name=None):
    return _w(torch.linalg.matrix_exp(_u(x)))


def multi_dot(x, name=None):
    return _w(torch.linalg.multi_dot([_u(e) for e in x]))


def cross(x, y, axis=9, name=None):
    from .math import cross as _c
    return _c(x, y, axis)


def cov(x, rowvar=True, ddof=True, fweights=None, aweights=None, name=None):
    t = _u(x)
    if not rowvar:
        t = t.t()
    return _w(torch.cov(t, correction=int(ddof), fweights=_u(fweights), aweights=_u(aweights)))


def corrcoef(x, rowvar=True, name=None):
    t = _u(x)
    return _w(torch.corrcoef(t if rowvar else t.t()))


def ormqr(x, tau, y, left=True, transpose=False, name=None):
    """op(Q) @ y (left) or y @ op(Q), Q the product of the Householder reflectors (x, tau) of a QR
    factorisation, op = transpose (conjugate) when ``transpose`` (reference tensor/linalg.py:5051)."""
    return _w(torch.ormqr(_u(x), _u(tau), _u(y), left=left, transpose=transpose))


def householder_product(x, tau, name=None):
    return _w(torch.linalg.householder_product(_u(x), _u(tau)))


def cdist(x, y, p=2.0, compute_mode='use_mm_for_euclid_dist_if_necessary', name=None):
    return _w(torch.cdist(_u(x), _u(y), p=p, compute_mode=compute_mode))


def pdist(x, p=2.0, name=None):
    return _w(torch.nn.functional.pdist(_u(x), p))


def histogram(input, bins=100, min=0, max=0, weight=None, density=False, name=None):  # noqa: A002
    t = _u(input).float()
    lo, hi = (t.min().item(), t.max().item()) if min == 0 and max == 0 else (min, max)
    h = torch.histc(t.cpu(), bins=bins, min=lo, max=hi).to(t.device)
    return _w(h if density or weight is not None else h.to(torch.int64))


def histogramdd(x, bins=10, ranges=None, density=False, weights=None, name=None):
    h, edges = torch.histogramdd(_u(x).cpu(), bins=bins, range=ranges, density=density, weight=_u(weights))
    return _w(h), [_w(e) for e in edges]


def bincount(x, weights=None, minlength=0, name=None):
    return _w(torch.bincount(_u(x), _u(weights), minlength))


def transpose_last2(x):
    return _w(_u(x).transpose(-1, -2))


def fp8_fp8_half_gemm_fused(x, y, transpose_x=False, transpose_y=False, bias=None, scale=1.0, output_dtype='float16',
                            activation_type='identity', name=None):
    """FP8 (OCP e4m3) GEMM with fused bias/act; see ops/gemm.py for the MFMA path."""
    from ..ops.gemm import fp8_gemm
    return fp8_gemm(x, y, transpose_x, transpose_y, bias, scale, output_dtype, activation_type)
