"""paddle.sparse (reference: python/paddle/sparse/{creation,unary,binary,multiary}.py).

COO and CSR tensors are torch sparse tensors (hipSPARSE kernels on the GPU) behind the same
``paddle.Tensor`` handle; elementwise unary ops act on the stored values only, so zeros stay
implicit.  Sparse convolutions / pooling live in ``paddle.sparse.nn`` (rulebook gather-GEMM-
scatter).
"""
import warnings

import numpy as np
import torch

from ..core.tensor import Tensor, _wrap, _unwrap
from ..core.dtype import to_torch_dtype
from . import nn  # noqa: F401

warnings.filterwarnings('ignore', message='Sparse CSR tensor support is in beta')


def _dev(place):
    from ..core.place import to_device
    return to_device(place)


def _arr(x, dtype=None, dev=None):
    if isinstance(x, Tensor):
        t = x._t
    elif isinstance(x, torch.Tensor):
        t = x
    else:
        a = np.asarray(x)
        if a.dtype == np.float64 and not isinstance(x, np.ndarray):
            a = a.astype(np.float32)  # python floats follow the default dtype
        t = torch.as_tensor(a)
    if dtype is not None:
        t = t.to(dtype)
    if dev is not None:
        t = t.to(dev)
    return t


def sparse_coo_tensor(indices, values, shape=None, dtype=None, place=None, stop_gradient=True):
    dev = _dev(place)
    idx = _arr(indices, torch.long, dev)
    vals = _arr(values, to_torch_dtype(dtype) if dtype is not None else None, dev)
    if shape is None:
        shape = (idx.max(1).values + 1).tolist() + list(vals.shape[1:])
    t = torch.sparse_coo_tensor(idx, vals, tuple(shape)).coalesce()
    if not stop_gradient:
        t.requires_grad_(True)
    return _wrap(t)


def sparse_csr_tensor(crows, cols, values, shape, dtype=None, place=None, stop_gradient=True):
    dev = _dev(place)
    t = torch.sparse_csr_tensor(_arr(crows, torch.long, dev), _arr(cols, torch.long, dev),
                                _arr(values, to_torch_dtype(dtype) if dtype is not None else None, dev), tuple(shape))
    if not stop_gradient:
        t.requires_grad_(True)
    return _wrap(t)


def _is_coo(t):
    return t.layout == torch.sparse_coo


def _is_csr(t):
    return t.layout == torch.sparse_csr


def _map_values(x, fn):
    t = _unwrap(x)
    if _is_coo(t):
        t = t.coalesce()
        return _wrap(torch.sparse_coo_tensor(t.indices(), fn(t.values()), t.shape))
    if _is_csr(t):
        return _wrap(torch.sparse_csr_tensor(t.crow_indices(), t.col_indices(), fn(t.values()), t.shape))
    return _wrap(fn(t))


def _unary(fn):
    def op(x, name=None):
        return _map_values(x, fn)
    return op


sin = _unary(torch.sin)
tan = _unary(torch.tan)
asin = _unary(torch.asin)
atan = _unary(torch.atan)
sinh = _unary(torch.sinh)
tanh = _unary(torch.tanh)
asinh = _unary(torch.asinh)
atanh = _unary(torch.atanh)
sqrt = _unary(torch.sqrt)
square = _unary(torch.square)
log1p = _unary(torch.log1p)
abs = _unary(torch.abs)  # noqa: A001
neg = _unary(torch.neg)
expm1 = _unary(torch.expm1)
deg2rad = _unary(torch.deg2rad)
rad2deg = _unary(torch.rad2deg)
isnan = _unary(torch.isnan)


def pow(x, factor, name=None):  # noqa: A001
    return _map_values(x, lambda v: v.pow(factor))


def cast(x, index_dtype=None, value_dtype=None, name=None):
    t = _unwrap(x)
    idt = to_torch_dtype(index_dtype) if index_dtype else None
    vdt = to_torch_dtype(value_dtype) if value_dtype else None
    if _is_coo(t):
        t = t.coalesce()
        i = t.indices() if idt is None else t.indices().to(idt)
        return _wrap(torch.sparse_coo_tensor(i, t.values().to(vdt) if vdt else t.values(), t.shape))
    return _map_values(x, lambda v: v.to(vdt) if vdt else v)


def _binary(fn):
    def op(x, y, name=None):
        a, b = _unwrap(x), _unwrap(y)
        csr = _is_csr(a)
        if csr:
            a = a.to_sparse_coo()
        if isinstance(b, torch.Tensor) and _is_csr(b):
            b = b.to_sparse_coo()
        out = fn(a, b)
        if out.layout == torch.sparse_coo:
            out = out.coalesce()
        return _wrap(out.to_sparse_csr() if csr and out.layout == torch.sparse_coo else out)
    return op


add = _binary(torch.add)
subtract = _binary(torch.sub)
multiply = _binary(torch.mul)


def divide(x, y, name=None):
    a, b = _unwrap(x), _unwrap(y)
    if isinstance(b, torch.Tensor) and b.layout != torch.strided:
        # same sparsity pattern: divide stored values
        a2, b2 = a.to_sparse_coo().coalesce(), b.to_sparse_coo().coalesce()
        out = torch.sparse_coo_tensor(a2.indices(), a2.values() / b2.values(), a.shape).coalesce()
        return _wrap(out.to_sparse_csr() if _is_csr(a) else out)
    return _map_values(x, lambda v: v / b)


def matmul(x, y, name=None):
    a, b = _unwrap(x), _unwrap(y)
    if a.layout != torch.strided and b.layout == torch.strided:
        return _wrap(torch.sparse.mm(a, b) if a.dim() == 2 else torch.bmm(a, b))
    return _wrap(torch.matmul(a, b))


def masked_matmul(x, y, mask, name=None):
    """(x @ y) sampled at the nonzeros of ``mask`` (SDDMM), returned in mask's layout."""
    a, b, m = _unwrap(x), _unwrap(y), _unwrap(mask)
    if _is_csr(m) and m.dim() == 2:
        zero = torch.sparse_csr_tensor(m.crow_indices(), m.col_indices(), torch.zeros_like(m.values()), m.shape)
        return _wrap(torch.sparse.sampled_addmm(zero, a, b, beta=0.0))
    mc = m.to_sparse_coo().coalesce()
    idx = mc.indices()
    if a.dim() == 2:
        vals = (a[idx[0]] * b.t()[idx[1]]).sum(-1)
    else:
        vals = (a[idx[0], idx[1]] * b.transpose(-1, -2)[idx[0], idx[2]]).sum(-1)
    out = torch.sparse_coo_tensor(idx, vals, mc.shape)
    return _wrap(out.to_sparse_csr() if _is_csr(m) else out)


def mv(x, vec, name=None):
    return _wrap(torch.mv(_unwrap(x), _unwrap(vec)))


def addmm(input, x, y, beta=1.0, alpha=1.0, name=None):  # noqa: A002
    return _wrap(torch.sparse.addmm(_unwrap(input), _unwrap(x), _unwrap(y), beta=beta, alpha=alpha)
                 if _unwrap(x).layout != torch.strided else
                 torch.addmm(_unwrap(input), _unwrap(x), _unwrap(y), beta=beta, alpha=alpha))


def transpose(x, perm, name=None):
    t = _unwrap(x)
    csr = _is_csr(t)
    c = t.to_sparse_coo().coalesce() if csr else t.coalesce()
    out = c.permute(*perm).coalesce()
    return _wrap(out.to_sparse_csr() if csr else out)


def reshape(x, shape, name=None):
    t = _unwrap(x)
    csr = _is_csr(t)
    d = t.to_dense().reshape(shape)
    return _wrap(d.to_sparse_csr() if csr else d.to_sparse(t.sparse_dim() if not csr else 2))


def sum(x, axis=None, dtype=None, keepdim=False, name=None):  # noqa: A001
    t = _unwrap(x)
    if axis is None:
        return _wrap(torch.sparse.sum(t.to_sparse_coo()) if t.layout != torch.strided else t.sum())
    out = torch.sparse.sum(t.to_sparse_coo(), dim=axis)
    if keepdim:
        out = out.to_dense().unsqueeze(axis).to_sparse()
    return _wrap(out)


def coalesce(x, name=None):
    return _wrap(_unwrap(x).coalesce())


def is_same_shape(x, y):
    return list(x.shape) == list(y.shape)


def mask_as(x, mask, name=None):
    d, m = _unwrap(x), _unwrap(mask)
    mc = m.to_sparse_coo().coalesce()
    idx = mc.indices()
    vals = d[tuple(idx)] if mc.sparse_dim() == d.dim() else d[tuple(idx)]
    out = torch.sparse_coo_tensor(idx, vals, d.shape).coalesce()
    return _wrap(out.to_sparse_csr() if _is_csr(m) else out)


def slice(x, axes, starts, ends, name=None):  # noqa: A001
    t = _unwrap(x)
    csr = _is_csr(t)
    d = t.to_dense()
    sl = [__import__('builtins').slice(None)] * d.dim()
    for a, s, e in zip(axes, starts, ends):
        sl[a] = __import__('builtins').slice(s, e)
    out = d[tuple(sl)]
    return _wrap(out.to_sparse_csr() if csr else out.to_sparse(t.sparse_dim()))


def pca_lowrank(x, q=None, center=True, niter=2, name=None):
    t = _unwrap(x)
    U, S, V = torch.pca_lowrank(t.to_dense() if t.layout != torch.strided else t, q=q, center=center, niter=niter)
    return _wrap(U), _wrap(S), _wrap(V)


# ---- Tensor methods for sparse handles
def _install():
    def indices(self):
        return _wrap(self._t.coalesce().indices())

    def values(self):
        t = self._t
        return _wrap(t.coalesce().values() if _is_coo(t) else t.values())

    def crows(self):
        return _wrap(self._t.crow_indices())

    def cols(self):
        return _wrap(self._t.col_indices())

    def nnz(self):
        t = self._t
        return int(t._nnz()) if t.layout != torch.strided else int((t != 0).sum())

    def to_dense(self):
        return _wrap(self._t.to_dense())

    def to_sparse_coo(self, sparse_dim=None):
        t = self._t
        if t.layout == torch.strided:
            return _wrap(t.to_sparse(sparse_dim or t.dim()))
        return _wrap(t.to_sparse_coo().coalesce())

    def to_sparse_csr(self):
        return _wrap(self._t.to_sparse_csr())

    for k, v in dict(indices=indices, values=values, crows=crows, cols=cols, nnz=nnz, to_dense=to_dense,
                     to_sparse_coo=to_sparse_coo, to_sparse_csr=to_sparse_csr).items():
        if not hasattr(Tensor, k):
            setattr(Tensor, k, v)


_install()

__all__ = ['sparse_coo_tensor', 'sparse_csr_tensor', 'sin', 'tan', 'asin', 'atan', 'sinh', 'tanh', 'asinh', 'atanh',
           'sqrt', 'square', 'log1p', 'abs', 'pow', 'pca_lowrank', 'cast', 'neg', 'deg2rad', 'rad2deg', 'expm1', 'mv',
           'matmul', 'mask_as', 'masked_matmul', 'addmm', 'add', 'subtract', 'transpose', 'sum', 'multiply', 'divide',
           'coalesce', 'is_same_shape', 'reshape', 'isnan', 'slice']
