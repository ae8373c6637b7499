"""Functional quasi-Newton minimisers: BFGS and L-BFGS with a strong-Wolfe line search.

Reference: python/paddle/incubate/optimizer/functional/bfgs.py:27 (minimize_bfgs),
lbfgs.py:27 (minimize_lbfgs), line_search.py:62 (strong_wolfe).  Same arguments and the same
returned tuples; the reference builds its loops from static-graph while_loop ops, here they are
plain eager loops over device tensors (the stopping tests read one scalar per iteration).

Algorithms: Nocedal & Wright, Numerical Optimization (2nd ed.): BFGS Alg. 6.1, L-BFGS two-loop
recursion Alg. 7.4/7.5, strong-Wolfe line search Alg. 3.5 with the zoom of Alg. 3.6 (cubic
interpolation of the bracket, bisection safeguard).
"""
import torch

from ...core.tensor import Tensor, _wrap

__all__ = ['minimize_bfgs', 'minimize_lbfgs']


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


def _check_dtype(dtype):
    if dtype not in ('float32', 'float64'):
        raise ValueError(f"The dtype must be 'float32' or 'float64', but the specified is {dtype}.")
    return torch.float32 if dtype == 'float32' else torch.float64


def _value_and_grad(f, x):
    x = x.detach().clone().requires_grad_(True)
    with torch.enable_grad():
        v = f(_wrap(x))
        vt = _t(v)
        if vt.numel() != 1:
            raise ValueError("objective_func must return a scalar")
        g, = torch.autograd.grad(vt.reshape(()), x)
    return vt.detach().reshape(()), g.detach()


def _cubic_min(a1, f1, g1, a2, f2, g2):
    """Minimiser of the cubic through (a1, f1, g1) and (a2, f2, g2), clamped to the interval."""
    d1 = g1 + g2 - 3.0 * (f1 - f2) / (a1 - a2)
    sq = d1 * d1 - g1 * g2
    lo, hi = min(a1, a2), max(a1, a2)
    if sq >= 0:
        d2 = sq ** 0.5
        if a1 > a2:
            d2 = -d2
        denom = g2 - g1 + 2.0 * d2
        if denom != 0:
            a = a2 - (a2 - a1) * (g2 + d2 - d1) / denom
            return min(max(a, lo), hi)
    return 0.5 * (lo + hi)


def strong_wolfe(f, xk, pk, fk, gk, max_iters=50, initial_step_length=1.0, c1=1e-4, c2=0.9, alpha_max=10.0,
                 tolerance_change=1e-9):
    """Step length a along pk with f(xk + a pk) <= fk + c1 a gk.pk and |grad.pk| <= c2 |gk.pk|.

    Returns (a, f_new, g_new, calls)."""
    d0 = float((gk * pk).sum())
    f0 = float(fk)
    calls = 0

    def phi(a):
        nonlocal calls
        calls += 1
        v, g = _value_and_grad(f, xk + a * pk)
        return float(v), float((g * pk).sum()), v, g

    a_prev, f_prev, d_prev = 0.0, f0, d0
    a = float(initial_step_length)
    best = None
    for i in range(max_iters):
        fa, da, v, g = phi(a)
        best = (a, v, g)
        if fa > f0 + c1 * a * d0 or (i > 0 and fa >= f_prev):
            return _zoom(phi, a_prev, f_prev, d_prev, a, fa, da, f0, d0, c1, c2, max_iters, tolerance_change,
                         calls_box=lambda: calls, fallback=best)
        if abs(da) <= -c2 * d0:
            return a, v, g, calls
        if da >= 0:
            return _zoom(phi, a, fa, da, a_prev, f_prev, d_prev, f0, d0, c1, c2, max_iters, tolerance_change,
                         calls_box=lambda: calls, fallback=best)
        a_prev, f_prev, d_prev = a, fa, da
        a = min(2.0 * a, alpha_max)
    return best[0], best[1], best[2], calls


def _zoom(phi, a_lo, f_lo, d_lo, a_hi, f_hi, d_hi, f0, d0, c1, c2, max_iters, tol, calls_box, fallback):
    best = fallback
    for _ in range(max_iters):
        if abs(a_hi - a_lo) < tol:
            break
        a = _cubic_min(a_lo, f_lo, d_lo, a_hi, f_hi, d_hi)
        # keep the trial away from the bracket ends (bisection safeguard)
        w = abs(a_hi - a_lo)
        lo, hi = min(a_lo, a_hi), max(a_lo, a_hi)
        if a - lo < 0.1 * w or hi - a < 0.1 * w:
            a = 0.5 * (a_lo + a_hi)
        fa, da, v, g = phi(a)
        best = (a, v, g)
        if fa > f0 + c1 * a * d0 or fa >= f_lo:
            a_hi, f_hi, d_hi = a, fa, da
        else:
            if abs(da) <= -c2 * d0:
                return a, v, g, calls_box()
            if da * (a_hi - a_lo) >= 0:
                a_hi, f_hi, d_hi = a_lo, f_lo, d_lo
            a_lo, f_lo, d_lo = a, fa, da
    return best[0], best[1], best[2], calls_box()


def _prepare(objective_func, initial_position, dtype, line_search_fn):
    if line_search_fn != 'strong_wolfe':
        raise NotImplementedError(f"Currently only support line_search_fn = 'strong_wolfe', but the specified "
                                  f"is '{line_search_fn}'")
    dt = _check_dtype(dtype)
    x0 = _t(initial_position)
    if not isinstance(initial_position, Tensor):
        raise TypeError("The type of 'initial_position' in minimize must be Tensor")
    if x0.dtype != dt:
        raise ValueError(f"initial_position dtype {x0.dtype} does not match dtype='{dtype}'")
    return x0.detach().clone(), dt


def minimize_bfgs(objective_func, initial_position, max_iters=50, tolerance_grad=1e-7, tolerance_change=1e-9,
                  initial_inverse_hessian_estimate=None, line_search_fn='strong_wolfe', max_line_search_iters=50,
                  initial_step_length=1.0, dtype='float32', name=None):
    """Returns (is_converge, num_func_calls, position, objective_value, objective_gradient,
    inverse_hessian_estimate) — reference bfgs.py:27."""
    xk, dt = _prepare(objective_func, initial_position, dtype, line_search_fn)
    n = xk.shape[0]
    eye = torch.eye(n, dtype=dt, device=xk.device)
    if initial_inverse_hessian_estimate is None:
        Hk = eye.clone()
    else:
        Hk = _t(initial_inverse_hessian_estimate).to(dt).clone()
        if not torch.allclose(Hk, Hk.t()) or not bool((torch.linalg.eigvalsh(Hk) > 0).all()):
            raise ValueError("The initial_inverse_hessian_estimate should be symmetric and positive definite")
    fk, gk = _value_and_grad(objective_func, xk)
    calls = 1
    converged = bool(gk.abs().max() < tolerance_grad)
    k = 0
    while not converged and k < max_iters:
        pk = -(Hk @ gk)
        a, f_new, g_new, c = strong_wolfe(objective_func, xk, pk, fk, gk, max_iters=max_line_search_iters,
                                          initial_step_length=initial_step_length)
        calls += c
        sk = a * pk
        yk = g_new - gk
        x_new = xk + sk
        k += 1
        rho_inv = float((yk * sk).sum())
        if rho_inv != 0.0:
            rho = 1.0 / rho_inv
            V = eye - rho * torch.outer(sk, yk)
            Hk = V @ Hk @ V.t() + rho * torch.outer(sk, sk)
        dx = float((x_new - xk).abs().max())
        df = float((f_new - fk).abs())
        xk, fk, gk = x_new, f_new, g_new
        if float(gk.abs().max()) < tolerance_grad:
            converged = True
            break
        if dx < tolerance_change or df < tolerance_change or a == 0.0:
            break  # stalled: not converged in the gradient sense
    return (_wrap(torch.tensor([converged])), _wrap(torch.tensor([calls], dtype=torch.int64)), _wrap(xk),
            _wrap(fk), _wrap(gk), _wrap(Hk))


def minimize_lbfgs(objective_func, initial_position, history_size=100, max_iters=50, tolerance_grad=1e-8,
                   tolerance_change=1e-8, initial_inverse_hessian_estimate=None, line_search_fn='strong_wolfe',
                   max_line_search_iters=50, initial_step_length=1.0, dtype='float32', name=None):
    """Returns (is_converge, num_func_calls, position, objective_value, objective_gradient) —
    reference lbfgs.py:27.  H0 is the given estimate (identity by default)."""
    xk, dt = _prepare(objective_func, initial_position, dtype, line_search_fn)
    n = xk.shape[0]
    H0 = None if initial_inverse_hessian_estimate is None else _t(initial_inverse_hessian_estimate).to(dt)
    if H0 is not None and (not torch.allclose(H0, H0.t()) or not bool((torch.linalg.eigvalsh(H0) > 0).all())):
        raise ValueError("The initial_inverse_hessian_estimate should be symmetric and positive definite")
    fk, gk = _value_and_grad(objective_func, xk)
    calls = 1
    S, Y, R = [], [], []
    converged = bool(gk.abs().max() < tolerance_grad)
    k = 0
    while not converged and k < max_iters:
        # two-loop recursion: q = H_k g
        q = gk.clone()
        alphas = []
        for s, y, rho in reversed(list(zip(S, Y, R))):
            al = rho * float((s * q).sum())
            alphas.append(al)
            q = q - al * y
        r = q if H0 is None else H0 @ q
        for (s, y, rho), al in zip(zip(S, Y, R), reversed(alphas)):
            be = rho * float((y * r).sum())
            r = r + s * (al - be)
        pk = -r
        a, f_new, g_new, c = strong_wolfe(objective_func, xk, pk, fk, gk, max_iters=max_line_search_iters,
                                          initial_step_length=initial_step_length)
        calls += c
        sk = a * pk
        yk = g_new - gk
        k += 1
        ys = float((yk * sk).sum())
        if ys != 0.0:
            S.append(sk)
            Y.append(yk)
            R.append(1.0 / ys)
            if len(S) > history_size:
                S.pop(0), Y.pop(0), R.pop(0)
        x_new = xk + sk
        dx = float((x_new - xk).abs().max())
        df = float((f_new - fk).abs())
        xk, fk, gk = x_new, f_new, g_new
        if float(gk.abs().max()) < tolerance_grad:
            converged = True
            break
        if dx < tolerance_change or df < tolerance_change or a == 0.0:
            break
    del n
    return (_wrap(torch.tensor([converged])), _wrap(torch.tensor([calls], dtype=torch.int64)), _wrap(xk),
            _wrap(fk), _wrap(gk))
