"""CPU restatement of the reference's step-size ALS eigen-solvers
(`src/tt_als.py:876-1499`) -- TEST INFRASTRUCTURE, checker only.

Local eigenproblems go to SciPy ARPACK (`eigsh`, shift-invert via `splu`) or `lobpcg`
exactly as the reference does; the MI355X product replaces them with device dense
(generalised) symmetric eigensolvers."""
import os
import time

import numpy as np
import scipy.linalg as sla
import scipy.sparse as sps
import scipy.sparse.linalg as spla

from . import tt as T
from .als import phi_bck_A, phi_fwd_A
from .tt import einsum

_DEBUG = bool(os.environ.get("TTIPM_EIG_DEBUG"))  # diagnostics: one line per local step-size solve


def _v0(x):
    """`src/tt_als.py:876-881`"""
    x = np.asarray(x).reshape(-1)
    s = np.linalg.norm(x, ord=np.inf)
    if (not np.isfinite(s)) or s == 0:
        return None
    return x / s


def _quiet(e):
    """`src/tt_als.py:884-893`"""
    quiet = [sla.LinAlgWarning, sla.LinAlgError, np.linalg.LinAlgError]
    for name in ("ArpackError", "ArpackNoConvergence"):
        cls = getattr(spla, name, None)
        if cls is not None:
            quiet.append(cls)
    if "could not broadcast input array" in str(e):
        return
    if not isinstance(e, tuple(quiet)):
        print(f"	Attention: {e}")


def _ncv(m, requested=32):
    m = int(max(3, m))
    req = int(requested) if np.isfinite(requested) else 32
    return min(m, max(3, min(req, 64)))


def _maxiter(m):
    return max(20, min(300, 5 * int(max(1, m))))


def _lobpcg_maxiter(m):
    return max(20, min(100, int(max(1, m))))


def _res_stalled(prev, res, tol):
    return np.isfinite(prev) and np.isfinite(res) and res <= 50 * tol and res >= 0.8 * prev


def _step_stalled(prev_step, step, prev_res, res, tol):
    if prev_step is None:
        return False
    sc = max(abs(step), abs(prev_step), 1.0)
    return abs(step - prev_step) <= max(10 * tol, 1e-12) * sc and _res_stalled(prev_res, res, tol)


def _eigsh_min_with_polish(M, eps, m, v0):
    ev, sol = spla.eigsh(M, tol=eps, k=1, ncv=_ncv(m), maxiter=_maxiter(m), which="SA", v0=v0)
    if np.linalg.norm(M @ sol - ev * sol) > eps:
        sigma = ev.squeeze()
        lu = spla.splu((M - sigma * sps.eye(M.shape[1], format=M.format)).tocsc())
        op = spla.LinearOperator(M.shape, matvec=lambda v: lu.solve(v))
        evs, sol = spla.eigsh(op, k=1, which="LM", v0=_v0(sol), ncv=_ncv(m), maxiter=_maxiter(m), tol=eps)
        ev = sigma + 1 / evs
    return ev, sol


def _add_kick(u, v, r_add=2):
    """`src/tt_als.py:1041-1046`"""
    old = u.shape[-1]
    uk = np.random.randn(u.shape[0], r_add)
    u, Rm = sla.qr(np.concatenate((u, uk), 1), check_finite=False, mode="economic", overwrite_a=True)
    return u, Rm[:, :old] @ v, u.shape[-1]


def _add_kick_rev(u, v, r_add=2):
    """`src/tt_als.py:1048-1053`"""
    old = v.shape[0]
    uk = np.random.randn(r_add, v.shape[-1])
    Rm, v = sla.rq(np.concatenate((v, uk), 0), check_finite=False, mode="economic", overwrite_a=True)
    return u @ Rm[:old], v, v.shape[0]


def _split_two_site(sol, sh, trunc_tol, max_rank, bwd):
    if bwd:
        u, s, v = sla.svd(sol.reshape(int(np.prod(sh[:2])), int(np.prod(sh[2:]))).T, full_matrices=False,
                          check_finite=False, overwrite_a=True, lapack_driver="gesvd")
        v = s.reshape(-1, 1) * v
        r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
        s1, s2, r = _add_kick_rev(v[:r].T, u[:, :r].T, 4)
        return s1.reshape(sh[0], sh[1], r), s2.reshape(r, sh[2], sh[3])
    s1, s, s2 = sla.svd(sol.reshape(int(np.prod(sh[:2])), int(np.prod(sh[2:]))), full_matrices=False,
                        check_finite=False, overwrite_a=True, lapack_driver="gesvd")
    r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
    s1 = s1[:, :r]
    s2 = s.reshape(-1, 1)[:r] * s2[:r]
    s1, s2, r = _add_kick(s1, s2, 4)
    return s1.reshape(sh[0], sh[1], r), s2.reshape(r, sh[2], sh[3])


def step_size_local_solve(p1, p2, XAX_k, A_k, A_kp1, XAX_k2, XDX_k, D_k, D_kp1, XDX_k2,
                          step, size_limit, trunc_tol, eps, max_rank, bwd=True):
    """`_step_size_local_solve` (`src/tt_als.py:931-1038`)."""
    if (not np.isfinite(step)) or step <= 0:
        return p1, p2, 0.0, np.inf
    prev = einsum("rny,ytR->rntR", p1, p2)
    sh = prev.shape
    m = int(np.prod(sh))
    prev = prev.reshape(-1, 1)
    if sh[0] * sh[-1] <= size_limit:
        D = sps.csr_matrix(einsum("lsr,smnk,kptS,LSR->lmpLrntR", XDX_k, D_k, D_kp1, XDX_k2).reshape(m, m))
        D = 0.5 * (D + D.T)
        A = sps.csr_matrix(einsum("lsr,smnk,kptS,LSR->lmpLrntR", XAX_k, A_k, A_kp1, XAX_k2).reshape(m, m))
        A = 0.5 * (A + A.T)
        M = (1 / step) * A + D
        try:
            ev, sol = _eigsh_min_with_polish(M, eps, m, _v0(prev))
        except Exception as e:
            _quiet(e)
            ev = prev.T @ (M @ prev)
            sol = prev
        sol /= np.linalg.norm(sol)
        step_in, branch, ev_in = step, "keep", float(np.ravel(ev)[0])
        if ev < 0:
            try:
                ev, sol = spla.eigsh(-D, M=A, tol=eps, k=1, ncv=_ncv(m), which="LA", maxiter=_maxiter(m), v0=_v0(sol))
                step = max(0, min(step, 1 / ev[0]))
                branch = f"gen lam={ev[0]:.12e}"
            except Exception as e:
                _quiet(e)
                sol = prev
                step *= (1 - eps)
                branch = f"fail {type(e).__name__}"
        if _DEBUG:
            print(f"  ora two-site bwd={bwd} m={m} sh={sh} ev={ev_in:.6e} step {step_in:.12e} -> {step:.12e} {branch}")
        ev = prev.T @ (((1 / step) * A + D) @ prev)
        old_res = np.linalg.norm(((1 / step) * A + D) @ prev - ev * prev)
    else:
        eA = "lsr,smnk,kptS,LSR,rntR->lmpL"

        def mvA(v):
            return einsum(eA, XAX_k, A_k, A_kp1, XAX_k2, v.reshape(*sh)).reshape(-1, 1).__iadd__(1e-12 * v.reshape(-1, 1))

        def mvD(v):
            return einsum(eA, XDX_k, D_k, D_kp1, XDX_k2, v.reshape(*sh)).reshape(-1, 1).__imul__(-1)

        A_op = spla.LinearOperator((m, m), matvec=mvA)
        D_op = spla.LinearOperator((m, m), matvec=mvD)
        AD_op = spla.LinearOperator((m, m), matvec=lambda v: (mvA(v) / step).__isub__(mvD(v)))
        try:
            ev, sol = spla.lobpcg(AD_op, prev, tol=eps, largest=False, maxiter=_lobpcg_maxiter(m))
        except Exception:
            ev = prev.T @ AD_op(prev)
            sol = prev
        sol /= np.linalg.norm(sol)
        if ev < 0:
            try:
                ev, sol = spla.lobpcg(D_op, sol, B=A_op, tol=eps, maxiter=_lobpcg_maxiter(m))
                step = max(0, min(step, 1 / ev[0]))
            except Exception as e:
                _quiet(e)
                sol = prev
                step *= (1 - eps)
        ev = prev.T @ AD_op(prev)
        old_res = np.linalg.norm(AD_op(prev).__isub__(ev * prev))
    sol /= np.linalg.norm(sol)
    s1, s2 = _split_two_site(sol, sh, trunc_tol, max_rank, bwd)
    return s1, s2, step, old_res


def step_size_local_solve_last(prev, XDX_k, Dk, XDX_k1, XAX_k, Ak, XAX_k1, dense, step, eps):
    """`_step_size_local_solve_last` (`src/tt_als.py:1056-1129`)."""
    if (not np.isfinite(step)) or step <= 0:
        return prev.reshape(-1, 1), 0.0, np.inf
    m = int(np.prod(prev.shape))
    if dense:
        prev = prev.reshape(-1, 1)
        D = sps.csr_matrix(einsum("lsr,smnS,LSR->lmLrnR", XDX_k, Dk, XDX_k1).reshape(m, m))
        A = sps.csr_matrix(einsum("lsr,smnS,LSR->lmLrnR", XAX_k, Ak, XAX_k1).reshape(m, m))
        M = (1 / step) * A + D
        try:
            ev, sol = _eigsh_min_with_polish(M, eps, m, _v0(prev))
        except Exception as e:
            _quiet(e)
            ev = prev.T @ ((1 / step) * A + D) @ prev
            sol = prev
        step_in, branch, ev_in = step, "keep", float(np.ravel(ev)[0])
        if ev < 0:
            try:
                ev, sol = spla.eigsh(-D, M=A, tol=eps, k=1, ncv=_ncv(m), which="LA", maxiter=_maxiter(m), v0=_v0(sol))
                step = max(0, min(step, 1 / ev[0]))
                branch = f"gen lam={ev[0]:.12e}"
            except Exception as e:
                _quiet(e)
                sol = prev
                step *= (1 - eps)
                branch = f"fail {type(e).__name__}"
        if _DEBUG:
            print(f"  ora one-site m={m} ev={ev_in:.6e} step {step_in:.12e} -> {step:.12e} {branch}")
        ev = prev.T @ ((1 / step) * A + D) @ prev
        old_res = np.linalg.norm(((1 / step) * A + D) @ prev - ev * prev)
    else:
        xs = prev.shape
        prev = prev.reshape(-1, 1)
        eA = "lsr,smnS,LSR,rnR->lmL"

        def mvA(v):
            return einsum(eA, XAX_k, Ak, XAX_k1, v.reshape(*xs)).reshape(-1, 1).__iadd__(1e-12 * v.reshape(-1, 1))

        def mvD(v):
            return einsum(eA, XDX_k, Dk, XDX_k1, v.reshape(*xs)).reshape(-1, 1).__imul__(-1)

        A_op = spla.LinearOperator((m, m), matvec=mvA)
        D_op = spla.LinearOperator((m, m), matvec=mvD)
        AD_op = spla.LinearOperator((m, m), matvec=lambda v: (mvA(v) / step).__isub__(mvD(v)))
        try:
            ev, sol = spla.lobpcg(AD_op, X=prev, tol=eps, largest=False, maxiter=_lobpcg_maxiter(m))
        except Exception:
            ev = prev.T @ AD_op(prev)
            sol = prev
        if ev < 0:
            try:
                ev, sol = spla.lobpcg(D_op, X=sol, B=A_op, tol=eps, maxiter=_lobpcg_maxiter(m))
                step = max(0, min(step, 1 / ev[0]))
            except Exception as e:
                _quiet(e)
                sol = prev
                step *= (1 - eps)
        ev = prev.T @ AD_op(prev)
        old_res = np.linalg.norm(AD_op(prev).__isub__(ev * prev))
    return sol.reshape(-1, 1), step, old_res


def max_generalised_eigen(A, Delta, x0=None, nswp=10, tol=1e-8, size_limit=256, verbose=False):
    """`tt_max_generalised_eigen` (`src/tt_als.py:1132-1283`): largest alpha with A + alpha*Delta >= 0."""
    if x0 is None:
        x = T.random_gaussian([2] * (len(A) - 1), (A[0].shape[2],))
    else:
        x = x0
    d = len(x)
    rx = np.array([1] + T.ranks(x) + [1])
    N = np.array([c.shape[1] for c in x])
    XAX = [np.ones((1, 1, 1))] + [None] * (d - 1) + [np.ones((1, 1, 1))]
    XDX = [np.ones((1, 1, 1))] + [None] * (d - 1) + [np.ones((1, 1, 1))]
    step = 1
    local_res = np.inf * np.ones((2, d - 1))
    max_rank = int(np.floor(2 ** (d / 2)))
    trunc_tol = tol / np.sqrt(d)
    prev_step = None
    prev_res = np.inf
    swp = 0

    def finish_fwd():
        nonlocal step
        for k in range(d):
            sol, step, _ = step_size_local_solve_last(x[k], XDX[k], Delta[k], XDX[k + 1], XAX[k], A[k], XAX[k + 1],
                                                      np.sqrt(rx[k] * rx[k + 1]) < size_limit, step, tol)
            sol = np.reshape(sol, (rx[k] * N[k], rx[k + 1]))
            if k < d - 1:
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True, lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = u[:, :r].reshape(rx[k], N[k], r)
                x[k + 1] = einsum("ij,jkl->ikl", v[:r, :], x[k + 1]).reshape(r, N[k + 1], rx[k + 2])
                rx[k + 1] = r
                XAX[k + 1] = phi_fwd_A(XAX[k], x[k], A[k], x[k])
                XDX[k + 1] = phi_fwd_A(XDX[k], x[k], Delta[k], x[k])
            else:
                x[k] = np.reshape(sol, (rx[k], N[k], rx[k + 1]))

    def finish_bck():
        nonlocal step
        for k in range(d - 1, -1, -1):
            sol, step, _ = step_size_local_solve_last(x[k], XDX[k], Delta[k], XDX[k + 1], XAX[k], A[k], XAX[k + 1],
                                                      np.sqrt(rx[k] * rx[k + 1]) < size_limit, step, tol)
            sol = np.reshape(sol, (rx[k], N[k] * rx[k + 1])).T
            if k > 0:
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True, lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = np.reshape(u[:, :r].T, (r, N[k], rx[k + 1]))
                x[k - 1] = einsum("rdc,cR->rdR", x[k - 1], v[:r].T)
                rx[k] = r
                XAX[k] = phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
                XDX[k] = phi_bck_A(XDX[k + 1], x[k], Delta[k], x[k])
            else:
                x[k] = np.reshape(sol, (rx[k], N[k], rx[k + 1]))

    for swp in range(nswp):
        zero = False
        for k in range(d - 1, 0, -1):
            if swp > 0:
                x[k - 1], x[k], step, res = step_size_local_solve(
                    x[k - 1], x[k], XAX[k - 1], A[k - 1], A[k], XAX[k + 1],
                    XDX[k - 1], Delta[k - 1], Delta[k], XDX[k + 1], step, size_limit, trunc_tol, tol, max_rank, bwd=True)
                local_res[0, k - 1] = res
                if step <= 0:
                    zero = True
                    break
            else:
                sol = np.reshape(x[k], (rx[k], N[k] * rx[k + 1])).T
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True, lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = np.reshape(u[:, :r].T, (r, N[k], rx[k + 1]))
                x[k - 1] = einsum("rdc,cR->rdR", x[k - 1], v[:r].T)
            rx[k] = x[k].shape[0]
            XAX[k] = phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
            XDX[k] = phi_bck_A(XDX[k + 1], x[k], Delta[k], x[k])
        if zero:
            break
        if np.max(local_res) < tol or swp == nswp - 1:
            finish_fwd()
            break
        for k in range(d - 1):
            x[k], x[k + 1], step, res = step_size_local_solve(
                x[k], x[k + 1], XAX[k], A[k], A[k + 1], XAX[k + 2],
                XDX[k], Delta[k], Delta[k + 1], XDX[k + 2], step, size_limit, trunc_tol, tol, max_rank, bwd=False)
            local_res[1, k] = res
            if step <= 0:
                zero = True
                break
            rx[k + 1] = x[k + 1].shape[0]
            XAX[k + 1] = phi_fwd_A(XAX[k], x[k], A[k], x[k])
            XDX[k + 1] = phi_fwd_A(XDX[k], x[k], Delta[k], x[k])
        if zero:
            break
        if np.max(local_res) < tol:
            finish_bck()
            break
        sres = np.max(local_res)
        if swp >= 2 and _step_stalled(prev_step, step, prev_res, sres, tol):
            break
        prev_step = step
        prev_res = sres
    max_res = np.max(local_res)
    x = T.normalise(x)
    if max_res > tol:
        print('\t Target Residual not reached!', flush=True)
        step *= (tol / max_res)
    return step, x


def _eigen_local_solve(p1, p2, XAX_k, A_k, A_kp1, XAX_k2, size_limit, trunc_tol, eps, disc, max_rank, bwd=True):
    """`src/tt_als.py:1286-1343`"""
    prev = einsum("rny,ytR->rntR", p1, p2)
    sh = prev.shape
    m = int(np.prod(sh))
    prev = prev.reshape(-1, 1)
    if prev.shape[0] * prev.shape[-1] <= size_limit:
        A = sps.csr_matrix(einsum("lsr,smnk,kptS,LSR->lmpLrntR", XAX_k, A_k, A_kp1, XAX_k2).reshape(m, m))
        A = 0.5 * (A.T + A)
        try:
            ev, sol = spla.eigsh(A, tol=eps, k=1, which="SA", ncv=_ncv(m, disc * m), maxiter=_maxiter(m), v0=_v0(prev))
        except Exception as e:
            _quiet(e)
            sol = prev
            ev = prev.T @ A @ prev
            disc = min(0.999, disc * 1.1)
        old_res = np.linalg.norm(ev * prev - A @ prev)
    else:
        eA = "lsr,smnk,kptS,LSR,rntR->lmpL"
        A_op = spla.LinearOperator((m, m), matvec=lambda v: einsum(eA, XAX_k, A_k, A_kp1, XAX_k2, v.reshape(*sh)).reshape(-1, 1))
        try:
            ev, sol = spla.lobpcg(A_op, X=prev, tol=eps, largest=False, maxiter=_lobpcg_maxiter(m))
        except Exception as e:
            _quiet(e)
            sol = prev
            ev = prev.T @ A_op(prev)
            disc = min(0.999, disc * 1.1)
        old_res = np.linalg.norm(ev * prev - A_op(prev))
    s1, s2 = _split_two_site(sol, sh, trunc_tol, max_rank, bwd)
    disc = max(0.1, disc * 0.999)
    return s1, s2, old_res, disc


def _eigen_local_solve_last(prev, XAX_k, A_k, XAX_k1, m, size_limit, eps):
    """`src/tt_als.py:1346-1389`"""
    if prev.shape[0] * prev.shape[-1] <= size_limit:
        prev = prev.reshape(-1, 1)
        A = sps.csr_matrix(einsum("lsr,smnS,LSR->lmLrnR", XAX_k, A_k, XAX_k1).reshape(m, m))
        try:
            ev, sol = _eigsh_min_with_polish(A, eps, m, _v0(prev))
        except Exception as e:
            _quiet(e)
            sol = prev
            ev = prev.T @ A @ prev
        return sol, np.linalg.norm(ev * prev - A @ prev)
    xs = prev.shape
    prev = prev.reshape(-1, 1)
    eA = "lsr,smnS,LSR,rnR->lmL"
    A_op = spla.LinearOperator((m, m), matvec=lambda v: einsum(eA, XAX_k, A_k, XAX_k1, v.reshape(*xs)).reshape(-1, 1))
    try:
        ev, sol = spla.lobpcg(A_op, X=prev, tol=eps, largest=False, maxiter=_lobpcg_maxiter(m))
    except Exception as e:
        _quiet(e)
        sol = prev
        ev = prev.T @ A_op(prev)
    return sol.reshape(-1, 1), np.linalg.norm(ev * prev - A_op(prev))


def min_eig(A, x0=None, nswp=10, tol=1e-8, size_limit=64, return_eig_val=False, verbose=False):
    """`tt_min_eig` (`src/tt_als.py:1392-1499`)."""
    if x0 is None:
        x = T.random_gaussian([2] * (len(A) - 1), (A[0].shape[2],))
    else:
        x = x0
    d = len(x)
    rx = np.array([1] + T.ranks(x) + [1])
    N = np.array([c.shape[1] for c in x])
    XAX = [np.ones((1, 1, 1))] + [None] * (d - 1) + [np.ones((1, 1, 1))]
    max_rank = int(np.floor(2 ** (d / 2)))
    trunc_tol = 0.1 * tol / np.sqrt(d)
    disc = 0.5
    prev_res = np.inf
    for swp in range(nswp):
        max_res = np.inf if swp == 0 else 0
        for k in range(d - 1, 0, -1):
            if swp > 0:
                x[k - 1], x[k], lr, disc = _eigen_local_solve(x[k - 1], x[k], XAX[k - 1], A[k - 1], A[k], XAX[k + 1],
                                                               size_limit, trunc_tol, tol, disc, max_rank, bwd=True)
                max_res = max(max_res, lr)
            else:
                sol = np.reshape(x[k], (rx[k], N[k] * rx[k + 1])).T
                u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True, lapack_driver="gesvd")
                v = s.reshape(-1, 1) * v
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = np.reshape(u[:, :r].T, (r, N[k], rx[k + 1]))
                x[k - 1] = einsum("rdc,cR->rdR", x[k - 1], v[:r].T)
            rx[k] = x[k].shape[0]
            XAX[k] = phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
        if max_res < tol or swp == nswp - 1:
            for k in range(d):
                sol, _ = _eigen_local_solve_last(x[k], XAX[k], A[k], XAX[k + 1], rx[k] * N[k] * rx[k + 1], size_limit, tol)
                sol = np.reshape(sol, (rx[k] * N[k], rx[k + 1]))
                if k < d - 1:
                    u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True, lapack_driver="gesvd")
                    v = s.reshape(-1, 1) * v
                    r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                    x[k] = u[:, :r].reshape(rx[k], N[k], r)
                    x[k + 1] = einsum("ij,jkl->ikl", v[:r, :], x[k + 1]).reshape(r, N[k + 1], rx[k + 2])
                    rx[k + 1] = r
                    XAX[k + 1] = phi_fwd_A(XAX[k], x[k], A[k], x[k])
                else:
                    x[k] = np.reshape(sol, (rx[k], N[k], rx[k + 1]))
            break
        max_res = 0
        for k in range(d - 1):
            x[k], x[k + 1], lr, disc = _eigen_local_solve(x[k], x[k + 1], XAX[k], A[k], A[k + 1], XAX[k + 2],
                                                           size_limit, trunc_tol, tol, disc, max_rank, bwd=False)
            max_res = max(max_res, lr)
            rx[k + 1] = x[k + 1].shape[0]
            XAX[k + 1] = phi_fwd_A(XAX[k], x[k], A[k], x[k])
        if max_res < tol:
            for k in range(d - 1, -1, -1):
                sol, _ = _eigen_local_solve_last(x[k], XAX[k], A[k], XAX[k + 1], rx[k] * N[k] * rx[k + 1], size_limit, tol)
                sol = np.reshape(sol, (rx[k], N[k] * rx[k + 1])).T
                if k > 0:
                    u, s, v = sla.svd(sol, full_matrices=False, check_finite=False, overwrite_a=True, lapack_driver="gesvd")
                    v = s.reshape(-1, 1) * v
                    r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                    x[k] = np.reshape(u[:, :r].T, (r, N[k], rx[k + 1]))
                    x[k - 1] = einsum("rdc,cR->rdR", x[k - 1], v[:r].T)
                    rx[k] = r
                    XAX[k] = phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
                else:
                    x[k] = np.reshape(sol, (rx[k], N[k], rx[k + 1]))
            break
        if swp >= 2 and _res_stalled(prev_res, max_res, tol):
            break
        prev_res = max_res
    x = T.normalise(x)
    mev = None
    if return_eig_val:
        mev = T.inner(x, T.fast_matrix_vec_mul(A, x, 1e-12))
    return x, mev
