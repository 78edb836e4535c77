"""Step-size ALS eigen-solvers on the MI355X -- drop-in for `tt_max_generalised_eigen`
(`src/tt_als.py:1132-1283`) and `tt_min_eig` (`:1392-1499`).

Environments and two-site local matrices are device contractions (MFMA GEMM steps).  The local
eigenproblems, which the reference sends to ARPACK `eigsh` (with an `splu` shift-invert polish)
or `lobpcg`, are solved exactly with the device extreme-eigenpair solver (`ttk_syev_extreme`); the
generalised problem `-D v = lambda A v` goes through a device Cholesky of A.  The converged
eigenpair is the same to the reference's tolerance (tol = 1e-8); ARPACK's failure branches
(exceptions) map to the same fallbacks."""
import os
import threading
import time

import numpy as np

from . import dev as D
from . import rng as _rng
from . import tt_als as _TA
from . import tt_ops as T
from .dev import einsum
from .tt_als import compute_phi_bck_A, compute_phi_fwd_A

TWO_SITE = "lsr,smnk,kptS,LSR->lmpLrntR"
ONE_SITE = "lsr,smnS,LSR->lmLrnR"
MAX_DENSE = 4096
_DEBUG = bool(os.environ.get("TTIPM_EIG_DEBUG"))
# normalisation / Rayleigh residual on the device with one (or no) host read; same arithmetic
_FUSED_TAIL = os.environ.get("TTIPM_EIG_FUSED_TAIL", "1") == "1"  # diagnostics: one line per local step-size solve
# tt_max_generalised_eigen's sweeps orchestrated in C++ (_ttkbind.eig_als, csrc/ttk_host_eig.inc): the
# same libttk calls in the same order as the Python below, bit-identical; "0" keeps the Python path
_NATIVE = os.environ.get("TTIPM_NATIVE_EIG", "1") == "1"
_NATIVE_BOUND = []


def _sym(Mt, m):
    M = Mt.view(m, m)
    if _FUSED_TAIL:  # (M + M^T) / 2 as clone + copy_(S, M^T, 0.5, 0.5), in one launch
        return D.axpby(M.t(), M, 0.5, 0.5, 1.0)
    S = D.clone(M)
    D.copy_(S, M.t(), 0.5, 0.5)
    return S


def _shifted(Am, Dm, step):
    """M = A / step + D (scaled + copy_, one launch)."""
    if _FUSED_TAIL:
        return D.axpby(Dm, Am, 1.0, 1.0, 1.0 / step)
    M = D.scaled(Am, 1.0 / step)
    D.copy_(M, Dm, 1.0, 1.0)
    return M


def _min_eigpair(M):
    return D.syev_extreme(M, largest=False)


def _gen_max_eig(Dm, Am):
    """largest lambda of -D v = lambda A v (eigsh(-D, M=A, which='LA')); raises if A not PD."""
    m = Am.shape[0]
    L = D.clone(Am)
    D.cholesky_(L)
    C = D.scaled(Dm, -1.0)
    D.trsm_(L, C)  # L^-1 (-D)
    Ct = D.clone(C.t())
    D.trsm_(L, Ct)  # L^-1 (L^-1 (-D))^T = L^-1 (-D) L^-T
    S = D.clone(Ct)
    D.copy_(S, Ct.t(), 0.5, 0.5)
    lam, w = D.syev_extreme(S, largest=True)
    y = w.view(m, 1)
    D.trsm_(L, y, trans=True)
    return lam, y.view(-1)


def _rayleigh(Am, Dm, step, v):
    """eig = v^T M v, res = ||M v - eig v|| for M = A/step + D."""
    M = _shifted(Am, Dm, step)
    Mv = D.matmul(M, v.view(-1, 1)).view(-1)
    if _FUSED_TAIL and v.is_contiguous():
        return D.rayleigh_tail_(v, Mv)
    ev = D.dot(v, Mv)
    D.copy_(Mv, v, -ev, 1.0)
    return ev, D.norm(Mv)


def _normalise(v):
    if _FUSED_TAIL:
        return D.normalized(v)
    return D.scaled(v, 1.0 / D.norm(v))


def _kick(u, v, r_add):
    """`_add_kick_rank` (`src/tt_als.py:1041-1046`)."""
    old = u.shape[-1]
    uk = D.from_numpy(_rng.R().randn(u.shape[0], r_add))
    cat = D.empty(u.shape[0], old + r_add)
    D.copy_(cat[:, :old], u)
    D.copy_(cat[:, old:], uk)
    q, Rm = D.qr(cat)
    return q, D.matmul(Rm[:, :old], v), q.shape[-1]


def _kick_rev(u, v, r_add):
    """`_add_kick_rank_rev` (`src/tt_als.py:1048-1053`)."""
    old = v.shape[0]
    uk = D.from_numpy(_rng.R().randn(r_add, v.shape[-1]))
    cat = D.empty(old + r_add, v.shape[-1])
    D.copy_(cat[:old], v)
    D.copy_(cat[old:], uk)
    Rm, q = D.rq(cat)
    return D.matmul(u, Rm[:old]), q, q.shape[0]


def _split_svd(sol, sh, bwd, S_out=None):
    """the SVD `_split` truncates (S into `S_out` without a host read when given)"""
    a, b = sh[0] * sh[1], sh[2] * sh[3]
    mat = D.clone(sol.view(a, b).t()) if bwd else sol.view(a, b)
    return D.svd(mat, host=S_out is None, S_out=S_out)


def _split(sol, sh, trunc_tol, max_rank, bwd, pre=None):
    """`pre`: the (U, S, Vt, s) of `_split_svd(sol, ...)` when already computed"""
    U, S, Vt, s = _split_svd(sol, sh, bwd) if pre is None else pre
    if bwd:
        v = einsum("r,rj->rj", S, Vt)
        r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
        s1, s2, r = _kick_rev(v[:r].t(), U[:, :r].t(), 4)  # strided operands: no transpose copies
        return D.contig(s1).view(sh[0], sh[1], r), D.contig(s2).view(r, sh[2], sh[3])
    r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
    s2 = einsum("r,rj->rj", S[:r], Vt[:r])
    s1, s2, r = _kick(U[:, :r], s2, 4)  # the kick copies the truncated factor itself
    return D.contig(s1).view(sh[0], sh[1], r), D.contig(s2).view(r, sh[2], sh[3])


def _check_dense(m):
    if m > MAX_DENSE:
        raise NotImplementedError(f"local eigenproblem of size {m} exceeds the dense device solver cap {MAX_DENSE}")


class LobpcgFailure(UserWarning):
    """scipy.sparse.linalg.lobpcg's UserWarnings (not converged / B-orthonormalisation failed), which
    the reference turns into exceptions (`warnings.simplefilter("error")`, src/tt_ipm.py:16)."""


def _lobpcg_maxiter(m):
    """`src/tt_als.py:907-909`"""
    return max(20, min(100, int(max(1, m))))


def lobpcg(A, x0, B=None, tol=1e-8, maxiter=20, largest=True, restart_control=20):
    """Single-vector LOBPCG on the device with scipy.sparse.linalg.lobpcg's control flow (scipy 1.15:
    B-orthonormalisation by Cholesky, implicit Gram blocks until the residual drops below
    sqrt(eps_mach), 3x3 Rayleigh-Ritz with a 2x2 restart, best-iterate return), used where the
    reference calls `scp.sparse.linalg.lobpcg` (`src/tt_als.py:1006,1013,1114,1120,1320,1382`).
    A, B: callables mapping a device vector (m,) to a new device vector.  The m-length work
    (operator applies, axpys, the 3x6 Gram block as one GEMM) stays on the device; the host solves
    the 3x3 pencil.  Non-convergence raises LobpcgFailure, as the reference's warnings do."""
    import scipy.linalg as sla
    m = x0.numel()
    V = D.empty(3, m)    # X, R, P
    W = D.empty(6, m)    # AX, AR, AP, BX, BR, BP
    X, R, P = V[0], V[1], V[2]
    AX, AR, AP, BX, BR, BP = W[0], W[1], W[2], W[3], W[4], W[5]

    def apply(op, src, dst):
        D.copy_(dst, op(src) if op is not None else src)

    D.copy_(X, x0.reshape(-1))
    apply(B, X, BX)
    vbv = D.dot(X, BX)
    if not vbv > 0:
        raise ValueError("Linearly dependent initial approximations")
    sc = 1.0 / np.sqrt(vbv)
    D.copy_(X, X, sc)
    D.copy_(BX, BX, sc)
    apply(A, X, AX)
    lam = D.dot(X, AX)
    best = D.clone(X)
    smallest = np.finfo(np.float64).max
    it, restart, forced, explicit, have_p = -1, True, False, False, False
    myeps = np.sqrt(np.finfo(np.float64).eps)
    rn = np.inf
    while it < maxiter:
        it += 1
        D.copy_(R, AX)
        D.copy_(R, BX, -lam, 1.0)
        rn = D.norm(R)
        if rn < smallest:
            smallest = rn
            D.copy_(best, X)
        elif rn > 2 ** restart_control * smallest:
            forced = True
            apply(A, X, AX)
            apply(B, X, BX)
        if not rn > tol:
            break
        D.copy_(R, X, -D.dot(BX, R), 1.0)  # R -= X (BX^T R)
        apply(B, R, BR)
        rbr = D.dot(R, BR)
        if not rbr > 0:
            raise LobpcgFailure(f"Failed at iteration {it} with accuracies {rn} not reaching the requested "
                                f"tolerance {tol}.")
        sc = 1.0 / np.sqrt(rbr)
        D.copy_(R, R, sc)
        D.copy_(BR, BR, sc)
        apply(A, R, AR)
        if it > 0:
            pbp = D.dot(P, BP)
            if pbp > 0:
                sc = 1.0 / np.sqrt(pbp)
                D.copy_(P, P, sc)
                D.copy_(BP, BP, sc)
                D.copy_(AP, AP, sc)
                restart = forced
            else:
                restart = True
        explicit = not (rn > myeps and not explicit)
        G = D.read(einsum("im,jm->ij", V, W))  # rows X,R,P; cols AX,AR,AP,BX,BR,BP
        xar, rar = G[0, 1], G[1, 1]
        if explicit:
            xax, xbx, rbr_, xbr = G[0, 0], G[0, 3], G[1, 4], G[0, 4]
        else:
            xax, xbx, rbr_, xbr = lam, 1.0, 1.0, 0.0
        ev_vec = None
        if not restart:
            xap, rap, pap, xbp, rbp = G[0, 2], G[1, 2], G[2, 2], G[0, 5], G[1, 5]
            pbp_ = G[2, 5] if explicit else 1.0
            gA = np.array([[xax, xar, xap], [xar, rar, rap], [xap, rap, pap]])
            gB = np.array([[xbx, xbr, xbp], [xbr, rbr_, rbp], [xbp, rbp, pbp_]])
            try:
                lams, vecs = sla.eigh(gA, gB, check_finite=False)
                ev_vec = vecs
            except np.linalg.LinAlgError:
                restart = True
        if restart:
            gA = np.array([[xax, xar], [xar, rar]])
            gB = np.array([[xbx, xbr], [xbr, rbr_]])
            try:
                lams, vecs = sla.eigh(gA, gB, check_finite=False)
                ev_vec = vecs
            except np.linalg.LinAlgError as e:
                raise LobpcgFailure(f"eigh failed at iteration {it} with error {e}")
        i = len(lams) - 1 if largest else 0
        lam = float(lams[i])
        c = ev_vec[:, i]
        cx, cr = float(c[0]), float(c[1])
        cp = float(c[2]) if not restart else 0.0
        # pp = R cr + P cp (likewise A-, B-images), X = X cx + pp, P = pp
        for vx, vr, vp in ((X, R, P), (AX, AR, AP), (BX, BR, BP)):
            if not restart:
                D.copy_(vp, vp, cp)
                D.copy_(vp, vr, cr, 1.0)
            else:
                D.copy_(vp, vr, cr)
            D.copy_(vx, vx, cx)
            D.copy_(vx, vp, 1.0, 1.0)
        have_p = True
    D.copy_(R, AX)
    D.copy_(R, BX, -lam, 1.0)
    rn = D.norm(R)
    if rn < smallest:
        smallest = rn
        D.copy_(best, X)
    if rn > tol:
        raise LobpcgFailure(f"Exited at iteration {it} with accuracies {rn} not reaching the requested "
                            f"tolerance {tol}.")
    return lam, best


class _Deferred:
    """Local residuals of one eigen-ALS half-sweep kept on the device: each dense local solve's
    Rayleigh tail writes (ev, ||r||^2) into a slot; the sweep only needs the residuals in
    np.max(local_res) after the half-sweep, so they are read there in ONE host wait instead of one
    per local solve (same values: the kernel is the one ttk_rayleigh_tail_sync runs)."""

    def __init__(self, cap):
        self.buf = D.empty(2 * max(cap, 1))
        self.n = 0
        self.pending = []  # (row, col, slot)

    def rayleigh(self, Am, Dm, step, v):
        M = _shifted(Am, Dm, step)
        Mv = D.matmul(M, v.view(-1, 1)).view(-1)
        if self.n * 2 + 2 > self.buf.numel():
            return _rayleigh(Am, Dm, step, v)[1]
        D.rayleigh_tail_into(v, Mv, self.buf[2 * self.n:2 * self.n + 2])
        self.n += 1
        return _Slot(self.n - 1)

    def put(self, arr, i, j, res):
        if isinstance(res, _Slot):
            self.pending.append((i, j, res.k))
        else:
            arr[i, j] = res

    def resolve(self, arr):
        if self.pending:
            h = D.read(self.buf[:2 * self.n])
            for i, j, k in self.pending:
                arr[i, j] = float(np.sqrt(max(h[2 * k + 1], 0.0)))
        self.pending, self.n = [], 0


class _Slot:
    def __init__(self, k):
        self.k = k


class _EigThread(threading.local):
    def __init__(self):
        self.defer = None  # the active _Deferred of tt_max_generalised_eigen's sweep, or "skip" (residual unused)
        self.min_eig_tol = 1e-8  # tt_min_eig's tolerance for the local LOBPCG solves


_ET = _EigThread()  # per host thread: several solves may run at once in one process


def _dense_step(prev, Am, Dm, step, eps, tag, post=None):
    """dense branch of the step-size local solves: M = A/step + D, smallest eigenpair; if negative,
    the largest lambda of -D v = lambda A v bounds the step (`src/tt_als.py:957-996,1060-1101`).

    `post` = (k, fn): the caller's next device step on the solution -- fn(sol, S_out) enqueues the
    truncation SVD (k singular values into S_out) and returns its (U, S, Vt, None).  It is enqueued
    speculatively right behind the eigensolve, on the branch taken when ev >= 0, and the eigenvalue
    and the k singular values come back in ONE host read; on ev < 0 that work is dropped (it has no
    side effects) and the caller redoes it on the branch's solution.  Returns (sol, step, residual,
    pre) with pre = the SVD tuple (host singular values filled in) or None."""
    M = _shifted(Am, Dm, step)
    pre = None
    if post is not None:
        k, fn = post
        comb = D.empty(1 + k)
        _, sol = D.syev_extreme(M, largest=False, lam_out=comb[:1])
        if tag == "two-site":
            sol = _normalise(sol)
        U, S, Vt, _ = fn(sol, comb[1:])
        h = D.read(comb)
        ev = float(h[0])
        if not ev < 0:
            pre = (U, S, Vt, h[1:])
    else:
        ev, sol = _min_eigpair(M)
        if tag == "two-site":
            sol = _normalise(sol)
    step_in, branch = step, "keep"
    if ev < 0:
        try:
            lam, sol = _gen_max_eig(Dm, Am)
            step = max(0, min(step, 1 / lam))
            branch = f"gen lam={lam:.12e}"
        except Exception as e:
            sol = prev
            step *= (1 - eps)
            branch = f"fail {type(e).__name__}"
    if _DEBUG:
        print(f"  dev {tag} m={prev.numel()} ev={ev:.6e} step {step_in:.12e} -> {step:.12e} {branch}")
    df = _ET.defer if _FUSED_TAIL and prev.is_contiguous() else None
    if df == "skip":  # the caller discards the residual: only its 1/step (ZeroDivisionError at 0) matters
        1.0 / step
        return sol, step, None, pre
    if df is not None:
        return sol, step, df.rayleigh(Am, Dm, step, prev), pre
    old_res = _rayleigh(Am, Dm, step, prev)[1]  # 1/step raises ZeroDivisionError at step 0, as the reference
    return sol, step, old_res, pre


def _iterative_step(prev, apply_A, apply_D, step, eps, tag):
    """LOBPCG branch of the step-size local solves (`src/tt_als.py:997-1021,1102-1127`):
    A_op = A + 1e-12 I, D_op = -D, AD_op = A_op/step - D_op (reads the current step)."""
    m = prev.numel()
    st = [step]

    def A_op(v):
        out = apply_A(v)
        D.copy_(out, v, 1e-12, 1.0)
        return out

    def D_op(v):
        return D.scaled(apply_D(v), -1.0)

    def AD_op(v):
        out = D.scaled(A_op(v), 1.0 / st[0])
        D.copy_(out, D_op(v), -1.0, 1.0)
        return out

    step_in, branch = step, "keep"
    try:
        ev, sol = lobpcg(AD_op, prev, tol=eps, largest=False, maxiter=_lobpcg_maxiter(m))
    except Exception as e:
        ev, sol = D.dot(prev, AD_op(prev)), prev
        branch = f"lobpcg-fail {type(e).__name__}"
    if tag == "two-site":
        sol = _normalise(sol)
    if ev < 0:
        try:
            lam, sol = lobpcg(D_op, sol, B=A_op, tol=eps, maxiter=_lobpcg_maxiter(m))
            st[0] = max(0, min(st[0], 1 / lam))
            branch = f"gen lam={lam:.12e}"
        except Exception as e:
            print(f"\tAttention: {e}")
            sol = prev
            st[0] *= (1 - eps)
            branch = f"gen-fail {type(e).__name__}"
    step = st[0]
    if _DEBUG:
        print(f"  dev {tag} lobpcg m={m} ev={ev:.6e} step {step_in:.12e} -> {step:.12e} {branch}")
    ADp = AD_op(prev)
    evp = D.dot(prev, ADp)
    D.copy_(ADp, prev, -evp, 1.0)
    return sol, step, D.norm(ADp)


def _step_size_local_solve(p1, p2, XAX_k, A_k, A_kp1, XAX_k2, XDX_k, D_k, D_kp1, XDX_k2, step, size_limit,
                           trunc_tol, eps, max_rank, bwd=True):
    """`_step_size_local_solve` (`src/tt_als.py:931-1038`): dense exact local eigensolve when
    r*R <= size_limit (the reference's ARPACK branch), device LOBPCG otherwise (its lobpcg branch)."""
    if (not np.isfinite(step)) or step <= 0:
        return p1, p2, 0.0, np.inf
    prev = einsum("rny,ytR->rntR", p1, p2)
    sh = tuple(prev.shape)
    m = int(np.prod(sh))
    if sh[0] * sh[-1] <= size_limit:
        _check_dense(m)
        pv = prev.view(-1)
        with D.einsum_batch():  # the two assemblies are independent: grouped launches, same arithmetic
            Dr = einsum(TWO_SITE, XDX_k, D_k, D_kp1, XDX_k2)
            Ar = einsum(TWO_SITE, XAX_k, A_k, A_kp1, XAX_k2)
        Dm, Am = _sym(Dr, m), _sym(Ar, m)
        k = min(sh[0] * sh[1], sh[2] * sh[3])
        sol, step, old_res, pre = _dense_step(
            pv, Am, Dm, step, eps, "two-site",
            post=(k, lambda v, S_out: _split_svd(_normalise(v), sh, bwd, S_out)) if _FUSED_TAIL else None)
        if pre is not None:
            s1, s2 = _split(None, sh, trunc_tol, max_rank, bwd, pre=pre)
            return s1, s2, step, old_res
    else:
        pv = prev.view(-1)
        eq = "lsr,smnk,kptS,LSR,rntR->lmpL"
        sol, step, old_res = _iterative_step(
            pv, lambda v: einsum(eq, XAX_k, A_k, A_kp1, XAX_k2, v.view(*sh)).view(-1),
            lambda v: einsum(eq, XDX_k, D_k, D_kp1, XDX_k2, v.view(*sh)).view(-1), step, eps, "two-site")
    sol = _normalise(sol)
    s1, s2 = _split(sol, sh, trunc_tol, max_rank, bwd)
    return s1, s2, step, old_res


def _step_size_local_solve_last(prev, XDX_k, Dk, XDX_k1, XAX_k, Ak, XAX_k1, dense, step, eps, post=None):
    """`_step_size_local_solve_last` (`src/tt_als.py:1056-1129`); `dense` is the reference's
    sqrt(r R) < size_limit flag.  Returns (sol, step, residual, pre): `post` / `pre` as in
    `_dense_step` (dense branch only; pre is None otherwise)."""
    if (not np.isfinite(step)) or step <= 0:
        return prev.reshape(-1) if prev.is_contiguous() else D.clone(prev).view(-1), 0.0, np.inf, None
    m = int(np.prod(prev.shape))
    xs = tuple(prev.shape)
    pv = D.contig(prev).view(-1)
    if dense:
        _check_dense(m)
        with D.einsum_batch():
            Dr = einsum(ONE_SITE, XDX_k, Dk, XDX_k1)
            Ar = einsum(ONE_SITE, XAX_k, Ak, XAX_k1)
        Dm, Am = _sym(Dr, m), _sym(Ar, m)
        return _dense_step(pv, Am, Dm, step, eps, "one-site", post=post if _FUSED_TAIL else None)
    eq = "lsr,smnS,LSR,rnR->lmL"
    return _iterative_step(pv, lambda v: einsum(eq, XAX_k, Ak, XAX_k1, v.view(*xs)).view(-1),
                           lambda v: einsum(eq, XDX_k, Dk, XDX_k1, v.view(*xs)).view(-1), step, eps,
                           "one-site") + (None,)


def _res_stalled(prev, res, tol):
    return np.isfinite(prev) and np.isfinite(res) and res <= 50 * tol and res >= 0.8 * prev


def _step_stalled(prev_step, step, prev_res, res, tol):
    if prev_step is None:
        return False
    sc = max(abs(step), abs(prev_step), 1.0)
    return abs(step - prev_step) <= max(10 * tol, 1e-12) * sc and _res_stalled(prev_res, res, tol)


def _svd_left(x, k, rx, N, trunc_tol, max_rank):
    """bck truncation of core k: returns (new core k, factor for core k-1 (R, rnew))."""
    mat = D.clone(D.contig(x[k]).view(rx[k], N[k] * rx[k + 1]).t())
    U, S, Vt, s = D.svd(mat)
    v = einsum("r,rj->rj", S, Vt)
    r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
    return D.clone(U[:, :r].t()).view(r, N[k], rx[k + 1]), v[:r], r


def _native_eig():
    """_ttkbind (with eig_als) when this call can run natively: the device path with the fused
    tails and environments, and no diagnostics that observe individual wrapper calls (FLOP
    counting, op statistics, fused-kernel checks, debug prints); else None."""
    B = D._BIND
    if not _NATIVE or B is None or not hasattr(B, "eig_als") or D.DEV.type != "cuda":
        return None
    if _DEBUG or not _FUSED_TAIL or not _TA.FUSED_ENV or D.ALGO is not None or D.OPSTATS is not None \
            or D._CHECK_FUSED or D._FUSED_ALL:
        return None
    if not _NATIVE_BOUND:
        import ctypes
        L = D.lib
        B.bind_eig([ctypes.cast(f, ctypes.c_void_p).value for f in (
            L.ttk_svd_work, L.ttk_svd_tol, L.ttk_qr_work, L.ttk_qr, L.ttk_syev_extreme_work, L.ttk_syev_extreme,
            L.ttk_read_sync, L.ttk_upload, L.ttk_cholesky_sync, L.ttk_trsm_lower, L.ttk_rayleigh_tail_dev,
            L.ttk_rayleigh_tail_sync, L.ttk_einsum_batch_begin, L.ttk_einsum_batch_end)
            + ((L.ttk_svd_tol_read,) if D._SVD_READ else ())])
        _NATIVE_BOUND.append(True)
    D._stream()
    D._fast()  # binds this thread's launch stream in the binder
    if D._TL.batch[0]:
        return None
    return B


# per process: how tt_max_generalised_eigen calls ran (native; python; native bail-outs to Python:
# a branch only Python takes, or a libttk failure the Python rerun reports with its own exception)
NATIVE_CALLS = {"native": 0, "python": 0, "bail": 0, "error": 0}


def tt_max_generalised_eigen(A, Delta, x0=None, nswp=10, tol=1e-8, size_limit=256, verbose=False):
    """`src/tt_als.py:1132-1283`: largest alpha with A + alpha*Delta >= 0 (two-site ALS)."""
    if verbose:
        print(f"\nStarting Eigen solve with:\n \t {tol} \n \t sweeps: {nswp}")
        t0 = time.time()
    x = T.tt_random_gaussian([2] * (len(A) - 1), (A[0].shape[2],)) if x0 is None else x0
    d = len(x)
    o3 = T._const("one111", np.ones((1, 1, 1)))
    B = _native_eig() if not verbose and d >= 2 else None
    if B is not None:
        # the sweeps below in C++; status 1 = a case only this Python handles (LOBPCG branch, dense cap,
        # a zero step): nothing was changed, rerun here from the same random state
        R = _rng.R()
        st = R.get_state()
        status, step, max_res, _, xs, key, pos, hg, g, why = B.eig_als(
            list(A), list(Delta), list(x), o3, int(nswp), float(tol), int(size_limit), float(tol / np.sqrt(d)),
            int(np.floor(2 ** (d / 2))), MAX_DENSE, st[1], st[2], st[3], st[4])
        if status == 0:
            NATIVE_CALLS["native"] += 1
            R.set_state(("MT19937", key, pos, hg, g))
            x[:] = xs
            max_res = np.float64(max_res)
            x = T.tt_normalise(x)
            if max_res > tol:
                print('\t Target Residual not reached!', flush=True)
                step *= (tol / max_res)
            return step, x
        NATIVE_CALLS["bail" if status == 1 else "error"] += 1
    NATIVE_CALLS["python"] += 1
    rx = np.array([1] + T.tt_ranks(x) + [1])
    N = np.array([c.shape[1] for c in x])
    XAX = [o3] + [None] * (d - 1) + [o3]
    XDX = [o3] + [None] * (d - 1) + [o3]
    step = 1
    local_res = np.inf * np.ones((2, d - 1))
    max_rank = int(np.floor(2 ** (d / 2)))
    trunc_tol = tol / np.sqrt(d)
    prev_step = None
    prev_res = np.inf
    swp = 0

    def finish_fwd():
        nonlocal step
        _ET.defer = "skip"  # the last local solves' residuals are discarded
        for k in range(d):
            a, b = rx[k] * N[k], rx[k + 1]
            post = (min(a, b), lambda v, S_out: D.svd(v.view(a, b), host=False, S_out=S_out)) if k < d - 1 else None
            sol, step, _, pre = _step_size_local_solve_last(x[k], XDX[k], Delta[k], XDX[k + 1], XAX[k], A[k],
                                                            XAX[k + 1], np.sqrt(rx[k] * rx[k + 1]) < size_limit,
                                                            step, tol, post)
            sol = sol.view(rx[k] * N[k], rx[k + 1])
            if k < d - 1:
                U, S, Vt, s = D.svd(sol) if pre is None else pre
                v = einsum("r,rj->rj", S, Vt)
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = D.clone(U[:, :r]).view(rx[k], N[k], r)
                x[k + 1] = einsum("ij,jkl->ikl", v[:r], x[k + 1])
                rx[k + 1] = r
                with D.einsum_batch():
                    XAX[k + 1] = compute_phi_fwd_A(XAX[k], x[k], A[k], x[k])
                    XDX[k + 1] = compute_phi_fwd_A(XDX[k], x[k], Delta[k], x[k])
            else:
                x[k] = D.contig(sol).view(rx[k], N[k], rx[k + 1])

    def finish_bck():
        nonlocal step
        _ET.defer = "skip"  # the last local solves' residuals are discarded
        for k in range(d - 1, -1, -1):
            a, b = rx[k], N[k] * rx[k + 1]
            post = (min(a, b), lambda v, S_out: D.svd(D.clone(v.view(a, b).t()), host=False, S_out=S_out)) \
                if k > 0 else None
            sol, step, _, pre = _step_size_local_solve_last(x[k], XDX[k], Delta[k], XDX[k + 1], XAX[k], A[k],
                                                            XAX[k + 1], np.sqrt(rx[k] * rx[k + 1]) < size_limit,
                                                            step, tol, post)
            if k > 0:
                if pre is None:
                    mat = D.clone(sol.view(rx[k], N[k] * rx[k + 1]).t())
                    U, S, Vt, s = D.svd(mat)
                else:
                    U, S, Vt, s = pre
                v = einsum("r,rj->rj", S, Vt)
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = D.clone(U[:, :r].t()).view(r, N[k], rx[k + 1])
                x[k - 1] = einsum("rdc,Rc->rdR", x[k - 1], v[:r])
                rx[k] = r
                with D.einsum_batch():
                    XAX[k] = compute_phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
                    XDX[k] = compute_phi_bck_A(XDX[k + 1], x[k], Delta[k], x[k])
            else:
                x[k] = D.contig(sol).view(rx[k], N[k], rx[k + 1])

    dfr = _Deferred(d)
    _ET.defer = dfr
    try:
        for swp in range(nswp):
            zero = False
            for k in range(d - 1, 0, -1):
                if swp > 0:
                    x[k - 1], x[k], step, res = _step_size_local_solve(
                        x[k - 1], x[k], XAX[k - 1], A[k - 1], A[k], XAX[k + 1], XDX[k - 1], Delta[k - 1], Delta[k],
                        XDX[k + 1], step, size_limit, trunc_tol, tol, max_rank, bwd=True)
                    dfr.put(local_res, 0, k - 1, res)
                    if step <= 0:
                        zero = True
                        break
                else:
                    x[k], vr, r = _svd_left(x, k, rx, N, trunc_tol, max_rank)
                    x[k - 1] = einsum("rdc,Rc->rdR", x[k - 1], vr)
                rx[k] = x[k].shape[0]
                XAX[k] = compute_phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
                XDX[k] = compute_phi_bck_A(XDX[k + 1], x[k], Delta[k], x[k])
            dfr.resolve(local_res)
            if zero:
                if verbose:
                    print("\tStep size reached zero; stopping eigen sweeps.", flush=True)
                break
            if np.max(local_res) < tol or swp == nswp - 1:
                finish_fwd()
                break
            if verbose:
                print('\tStarting Sweep: %d' % swp)
                print('\tStep size: %f' % step)
                print(f'\tResidual {np.max(local_res[0])}')
            for k in range(d - 1):
                x[k], x[k + 1], step, res = _step_size_local_solve(
                    x[k], x[k + 1], XAX[k], A[k], A[k + 1], XAX[k + 2], XDX[k], Delta[k], Delta[k + 1], XDX[k + 2],
                    step, size_limit, trunc_tol, tol, max_rank, bwd=False)
                dfr.put(local_res, 1, k, res)
                if step <= 0:
                    zero = True
                    break
                rx[k + 1] = x[k + 1].shape[0]
                XAX[k + 1] = compute_phi_fwd_A(XAX[k], x[k], A[k], x[k])
                XDX[k + 1] = compute_phi_fwd_A(XDX[k], x[k], Delta[k], x[k])
            dfr.resolve(local_res)
            if zero:
                if verbose:
                    print("\tStep size reached zero; stopping eigen sweeps.", flush=True)
                break
            if np.max(local_res) < tol:
                finish_bck()
                break
            sres = np.max(local_res)
            if swp >= 2 and _step_stalled(prev_step, step, prev_res, sres, tol):
                if verbose:
                    print("\tEigen sweep stalled; stopping early.", flush=True)
                break
            prev_step = step
            prev_res = sres
    finally:
        _ET.defer = None
    max_res = np.max(local_res)
    x = T.tt_normalise(x)
    if verbose:
        print(f"\t Solution rank is {rx[1:-1]}\n\t Step size: {step:f}\n\t Residual {max_res}")
        print('\t Number of sweeps', swp + 1, '\n\t Time: ', time.time() - t0, flush=True)
    if max_res > tol:
        print('\t Target Residual not reached!', flush=True)
        step *= (tol / max_res)
    return step, x


def _min_lobpcg(apply_A, prev):
    """`lobpcg(A_op, X=prev, tol, largest=False)` with the reference's fallback to prev."""
    m = prev.numel()
    try:
        return lobpcg(apply_A, prev, tol=_ET.min_eig_tol, largest=False, maxiter=_lobpcg_maxiter(m))
    except Exception as e:
        if not isinstance(e, LobpcgFailure):
            print(f"\tAttention: {e}")
        return D.dot(prev, apply_A(prev)), prev




def _eigen_local_solve(p1, p2, XAX_k, A_k, A_kp1, XAX_k2, size_limit, trunc_tol, max_rank, bwd=True):
    """`_eigen_local_solve` (`src/tt_als.py:1286-1343`): dense device eigensolve when
    m <= size_limit (the reference's eigsh branch), device LOBPCG otherwise."""
    prev = einsum("rny,ytR->rntR", p1, p2)
    sh = tuple(prev.shape)
    m = int(np.prod(sh))
    prev = prev.view(-1)
    if m <= size_limit:
        _check_dense(m)
        Am = _sym(einsum(TWO_SITE, XAX_k, A_k, A_kp1, XAX_k2), m)
        ev, sol = _min_eigpair(Am)
        Ap = D.matmul(Am, prev.view(-1, 1)).view(-1)
    else:
        eq = "lsr,smnk,kptS,LSR,rntR->lmpL"

        def apply_A(v):
            return einsum(eq, XAX_k, A_k, A_kp1, XAX_k2, v.view(*sh)).view(-1)
        ev, sol = _min_lobpcg(apply_A, prev)
        Ap = apply_A(prev)
    D.copy_(Ap, prev, ev, -1.0)  # ev*prev - A prev
    old_res = D.norm(Ap)
    s1, s2 = _split(sol, sh, trunc_tol, max_rank, bwd)
    return s1, s2, old_res


def _eigen_local_solve_last(prev, XAX_k, A_k, XAX_k1, m, size_limit):
    """`_eigen_local_solve_last` (`src/tt_als.py:1346-1389`): dense when r*R <= size_limit."""
    xs = tuple(prev.shape)
    dense = xs[0] * xs[-1] <= size_limit
    prev = D.contig(prev).view(-1)
    if dense:
        _check_dense(m)
        Am = _sym(einsum(ONE_SITE, XAX_k, A_k, XAX_k1), m)
        ev, sol = _min_eigpair(Am)
        return sol
    eq = "lsr,smnS,LSR,rnR->lmL"
    ev, sol = _min_lobpcg(lambda v: einsum(eq, XAX_k, A_k, XAX_k1, v.view(*xs)).view(-1), prev)
    return sol


def tt_min_eig(A, x0=None, nswp=10, tol=1e-8, size_limit=64, return_eig_val=False, verbose=False):
    """`tt_min_eig` (`src/tt_als.py:1392-1499`)."""
    x = T.tt_random_gaussian([2] * (len(A) - 1), (A[0].shape[2],)) if x0 is None else x0
    d = len(x)
    rx = np.array([1] + T.tt_ranks(x) + [1])
    N = np.array([c.shape[1] for c in x])
    o3 = T._const("one111", np.ones((1, 1, 1)))
    XAX = [o3] + [None] * (d - 1) + [o3]
    max_rank = int(np.floor(2 ** (d / 2)))
    trunc_tol = 0.1 * tol / np.sqrt(d)
    prev_res = np.inf
    _ET.min_eig_tol = tol

    def finish_fwd():
        for k in range(d):
            sol = _eigen_local_solve_last(x[k], XAX[k], A[k], XAX[k + 1], int(rx[k] * N[k] * rx[k + 1]), size_limit)
            sol = sol.view(rx[k] * N[k], rx[k + 1])
            if k < d - 1:
                U, S, Vt, s = D.svd(sol)
                v = einsum("r,rj->rj", S, Vt)
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = D.clone(U[:, :r]).view(rx[k], N[k], r)
                x[k + 1] = einsum("ij,jkl->ikl", v[:r], x[k + 1])
                rx[k + 1] = r
                XAX[k + 1] = compute_phi_fwd_A(XAX[k], x[k], A[k], x[k])
            else:
                x[k] = D.contig(sol).view(rx[k], N[k], rx[k + 1])

    def finish_bck():
        for k in range(d - 1, -1, -1):
            sol = _eigen_local_solve_last(x[k], XAX[k], A[k], XAX[k + 1], int(rx[k] * N[k] * rx[k + 1]), size_limit)
            if k > 0:
                mat = D.clone(sol.view(rx[k], N[k] * rx[k + 1]).t())
                U, S, Vt, s = D.svd(mat)
                v = einsum("r,rj->rj", S, Vt)
                r = min(T.prune_singular_vals(s, trunc_tol), max_rank)
                x[k] = D.clone(U[:, :r].t()).view(r, N[k], rx[k + 1])
                x[k - 1] = einsum("rdc,Rc->rdR", x[k - 1], v[:r])
                rx[k] = r
                XAX[k] = compute_phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
            else:
                x[k] = D.contig(sol).view(rx[k], N[k], rx[k + 1])

    for swp in range(nswp):
        max_res = np.inf if swp == 0 else 0
        for k in range(d - 1, 0, -1):
            if swp > 0:
                x[k - 1], x[k], lr = _eigen_local_solve(x[k - 1], x[k], XAX[k - 1], A[k - 1], A[k], XAX[k + 1],
                                                        size_limit, trunc_tol, max_rank, bwd=True)
                max_res = max(max_res, lr)
            else:
                x[k], vr, r = _svd_left(x, k, rx, N, trunc_tol, max_rank)
                x[k - 1] = einsum("rdc,Rc->rdR", x[k - 1], vr)
            rx[k] = x[k].shape[0]
            XAX[k] = compute_phi_bck_A(XAX[k + 1], x[k], A[k], x[k])
        if max_res < tol or swp == nswp - 1:
            finish_fwd()
            break
        max_res = 0
        for k in range(d - 1):
            x[k], x[k + 1], lr = _eigen_local_solve(x[k], x[k + 1], XAX[k], A[k], A[k + 1], XAX[k + 2],
                                                    size_limit, trunc_tol, max_rank, bwd=False)
            max_res = max(max_res, lr)
            rx[k + 1] = x[k + 1].shape[0]
            XAX[k + 1] = compute_phi_fwd_A(XAX[k], x[k], A[k], x[k])
        if max_res < tol:
            finish_bck()
            break
        if swp >= 2 and _res_stalled(prev_res, max_res, tol):
            break
        prev_res = max_res
    x = T.tt_normalise(x)
    mev = None
    if return_eig_val:
        mev = T.tt_inner_prod(x, T.tt_fast_matrix_vec_mul(A, x, 1e-12))
    return x, mev
