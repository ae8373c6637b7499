"""paddle.linalg (reference: python/paddle/linalg.py)."""
from .tensor.linalg import (cholesky, cholesky_solve, cholesky_inverse, norm, vector_norm, matrix_norm, cond, cov,  # noqa: F401
                            corrcoef, inv, eig, eigvals, eigh, eigvalsh, multi_dot, matrix_rank, svd, svdvals, qr,
                            lu, lu_unpack, matrix_power, matrix_exp, det, slogdet, pinv, solve, triangular_solve,
                            lstsq, householder_product, ormqr, svd_lowrank, pca_lowrank)
from .tensor.linalg import matmul, dot, mv, bmm, mm  # noqa: F401
