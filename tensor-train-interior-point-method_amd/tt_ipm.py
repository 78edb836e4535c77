"""TT-IPM on the MI355X -- drop-in for `src/tt_ipm.py` (same entry point `tt_ipm`, same
control flow and status fields).  The Newton/KKT hot path underneath (local KKT solves, AMEn,
rounding, zip-up products, step-size eigen solves) runs in libttk HIP kernels; this module keeps
the reference's host-side decisions.

Local KKT solvers (`_ipm_local_solver`, `src/tt_ipm.py:183-282`; `_ipm_local_solver_ineq`,
`:284-401`): dense Schur path = device assembly (MFMA GEMM), Cholesky, triangular solves, GEMMs
and LU with the scipy rcond warning rule; iterative path = device LGMRES (PETSc semantics) on
the Schur-reduced operator of `MatVecWrapper` (`cy_src/lgmres_cy.pyx:291-331`)."""
import ctypes
import os
import sys
import traceback
from dataclasses import dataclass
from enum import Enum

import time

import numpy as np

from . import dev as D
from . import rng as _rng
from ._lib import lib
from . import tt_ops as T
from .dev import einsum
from .lgmres import lgmres
from .tt_als import (TTBlockMatrix, TTBlockVector, _tt_get_block, tt_mat_mat_mul, tt_mat_vec_mul,
                     tt_restarted_block_amen)
from .tt_eig import tt_max_generalised_eigen, tt_min_eig

APPLY = "lsr,smnS,LSR,rnR->lmL"
APPLY_T = "lsr,smnS,LSR,lmL->rnR"
ASSEMBLE = "lsr,smnS,LSR->lmLrnR"
DIAG = "lsr,smnS,LSR->lmL"
RHS = "br,bmB,BR->rmR"

# True reproduces the shipped reference bug (cy_src/lgmres_cy.pyx:510): the first iterative
# inequality local solve raises.  Default: fixed (SURVEY.md §7 hard part 6).
INEQ_MATVEC_BUG = False

# LGMRES operator applies run as one fused launch each (Krylov iterates at rtol 1e-5 are insensitive
# to the association order; the AMEn residuals keep the reference's pairwise order)
FUSED_MATVEC = os.environ.get("TTIPM_FUSED_MATVEC", "1") == "1"
# ... and the whole Schur matvec as one native operator (2 launches per matvec, same arithmetic)
SCHUR_OP = os.environ.get("TTIPM_SCHUR_OP", "1") == "1"
# the dense Schur local solve as one library call (ttk_dense_schur_solve, bit-identical launches)
NATIVE_DENSE = os.environ.get("TTIPM_NATIVE_DENSE", "1") == "1"


class IneqMatvecBug(TypeError):
    pass


class MatVecWrapper:
    """Schur-reduced local KKT operator on [y; x] (`cy_src/lgmres_cy.pyx:203-331`):
    [B00 y + B01 x ; B21 x - B22 (invI o B01^T y)]."""

    keys = ((0, 0), (0, 1), (2, 1), (2, 2))

    def __init__(self, L, A, R, inv_I, shape):
        self.L = {k: L[k] for k in self.keys}
        self.A = {k: A[k] for k in self.keys}
        self.R = {k: R[k] for k in self.keys}
        self.inv_I = inv_I
        self.shape = shape
        r, n, RR = shape
        self.m = r * n * RR
        self.tmp = D.empty(r, n, RR)
        self.h = 0
        if FUSED_MATVEC and SCHUR_OP and not INEQ_MATVEC_BUG:
            order = [(0, 0), (0, 1), (2, 1), (2, 2), (0, 1)] + ([(3, 1), (3, 3)] if len(self.keys) > 4 else [])
            desc = []
            for k in order:
                desc += D.apply_desc(self.L[k], self.A[k], self.R[k], shape)
            h = ctypes.c_int64(0)
            arr = (ctypes.c_int64 * len(desc))(*desc)
            D._stream()
            self._ctx = D.ctx()
            D.check(lib.ttk_schur_build(self._ctx, int(len(self.keys) > 4), self.m, arr,
                                        inv_I.contiguous().data_ptr(), ctypes.byref(h)), "schur_build")
            self.h = h.value
            self._inv = inv_I  # keep the operands alive while the handle exists

    def __del__(self):
        if getattr(self, "h", 0):
            try:
                lib.ttk_schur_free(self._ctx, self.h)
            except Exception:
                pass

    def _parts(self, v, nb):
        r, n, R = self.shape
        return [v[i * self.m:(i + 1) * self.m].view(r, n, R) for i in range(nb)]

    def _op(self, key, v, out, alpha=1.0, beta=0.0):
        einsum(APPLY, self.L[key], self.A[key], self.R[key], v, out=out, alpha=alpha, beta=beta, fused=FUSED_MATVEC)

    def _schur_x(self, y):
        einsum(APPLY_T, self.L[0, 1], self.A[0, 1], self.R[0, 1], y, out=self.tmp, fused=FUSED_MATVEC)
        D.mul_(self.tmp, self.tmp, self.inv_I)
        return self.tmp

    def mv_flops(self):
        """Algorithmic FLOPs of one operator application (SURVEY.md §8(d) convention): the local
        applies it chains (`cy_src/lgmres_cy.pyx:297-327`: 5 blocks; 7 for the 3-block operator)."""
        if getattr(self, "_mvf", None) is None:
            sh = tuple(self.shape)
            blocks = [(APPLY, k) for k in self.keys] + [(APPLY_T, (0, 1))]
            self._mvf = sum(D.algo_flops(eq, (tuple(self.L[k].shape), tuple(self.A[k].shape),
                                              tuple(self.R[k].shape), sh)) for eq, k in blocks)
        return self._mvf

    def matvec_into(self, v, out):
        if self.h:
            D.count_algo(self.mv_flops() if D.ALGO is not None else 0.0, what="schur_matvec")
            D._stream()
            D.check(lib.ttk_schur_apply(self._ctx, self.h, v.data_ptr(), out.data_ptr()), "schur_apply")
            return out
        y, x = self._parts(v, 2)
        o0, o1 = self._parts(out, 2)
        self._op((0, 0), y, o0)
        self._op((0, 1), x, o0, beta=1.0)
        self._op((2, 1), x, o1)
        self._op((2, 2), self._schur_x(y), o1, alpha=-1.0, beta=1.0)
        return out

    def matvec(self, v):
        out = D.empty(v.numel())
        return self.matvec_into(v, out)


class IneqMatVecWrapper(MatVecWrapper):
    """`cy_src/lgmres_cy.pyx:379-510` on [y; x; t] (with the :510 bug fixed unless INEQ_MATVEC_BUG)."""

    keys = ((0, 0), (0, 1), (2, 1), (2, 2), (3, 1), (3, 3))

    def matvec_into(self, v, out):
        if INEQ_MATVEC_BUG:
            raise IneqMatvecBug("reference bug: IneqMatVecWrapper.matvec returns a memoryview")
        if self.h:
            D.count_algo(self.mv_flops() if D.ALGO is not None else 0.0, what="schur_matvec")
            D._stream()
            D.check(lib.ttk_schur_apply(self._ctx, self.h, v.data_ptr(), out.data_ptr()), "schur_apply")
            return out
        y, x, t = self._parts(v, 3)
        o0, o1, o2 = self._parts(out, 3)
        self._op((0, 0), y, o0)
        self._op((0, 1), x, o0, beta=1.0)
        self._op((2, 1), x, o1)
        w = self._schur_x(y)
        D.copy_(w, t, 1.0, 1.0)
        self._op((2, 2), w, o1, alpha=-1.0, beta=1.0)
        self._op((3, 1), x, o2)
        self._op((3, 3), t, o2, beta=1.0)
        return out


def _report(e):
    tb = traceback.extract_tb(e.__traceback__)
    last = tb[-1] if tb else None
    if last is None:
        print(f"\t⚠️ {type(e).__name__}: {e}")
    else:
        print(f"\t⚠️ {type(e).__name__} in {last.filename},\n\tline {last.lineno}: {last.line.strip()}")


def _local_rhs(Xb_k, b_k, Xb_k1, shape, nb):
    rhs = D.zeros(*shape)
    with D.einsum_batch():  # the blocks' contractions are independent: grouped launches, same arithmetic
        for i in range(nb):
            if i in b_k:
                einsum(RHS, Xb_k[i], b_k[i], Xb_k1[i], out=rhs[:, i])
    return rhs


def _residual_norm(A_k, XAX_k, XAX_k1, x, rhs, nrhs, res_out=None):
    """||A x - rhs|| / nrhs; with `res_out` (a device slice of length 1) ||A x - rhs||^2 is left there
    unread (the caller reads it together with later device scalars) and None is returned."""
    res = D.scaled(rhs, -1.0)
    A_k.block_local_product(XAX_k, XAX_k1, x, out=res)
    if res_out is not None:
        D.dot_into(res, res, res_out)
        return None
    return D.norm(res) / nrhs


def _rhs_and_residual_dots(A_k, XAX_k, XAX_k1, x, rhs, buf):
    """<rhs, rhs> and ||A x - rhs||^2 into the device slots buf[0:2] (no host read)."""
    D.dot_into(rhs, rhs, buf[0:1])
    res = D.scaled(rhs, -1.0)
    A_k.block_local_product(XAX_k, XAX_k1, x, out=res)
    D.dot_into(res, res, buf[1:2])


def _norms_from_dots(v):
    nrhs = max(D.norm_of(v[0]), 1e-10)
    return nrhs, D.norm_of(v[1]) / nrhs


def _rhs_and_residual_norms(A_k, XAX_k, XAX_k1, x, rhs):
    """(max(||rhs||, 1e-10), ||A x - rhs|| / that) with ONE host read (both dots on the device)."""
    buf = D.empty(2)
    _rhs_and_residual_dots(A_k, XAX_k, XAX_k1, x, rhs, buf)
    return _norms_from_dots(D.read(buf))


def _assemble(XAX_k, A_k, XAX_k1, key, m):
    return einsum(ASSEMBLE, XAX_k[key], A_k[key], XAX_k1[key]).view(m, m)


class _LocalBlock(ctypes.Structure):
    _fields_ = [("L", ctypes.c_void_p), ("A", ctypes.c_void_p), ("R", ctypes.c_void_p), ("s", ctypes.c_int64),
                ("S", ctypes.c_int64), ("a_strides", ctypes.c_int64 * 4)]


_TTK_ILL_CONDITIONED = 6


def _dense_native(XAX_k, A_k, XAX_k1, rhs, inv_I, xs):
    """`ttk_dense_schur_solve`: the dense branch below in one library call; its status maps onto
    the exceptions the Python steps raise (LinAlgError, LinAlgWarning-as-error)."""
    r, n, R = xs[0], xs[2], xs[3]
    arr = (_LocalBlock * 4)()
    keep = []
    for e, key in zip(arr, ((0, 0), (0, 1), (2, 1), (2, 2))):
        L, A, Rr = D.contig(XAX_k[key]), A_k[key], D.contig(XAX_k1[key])
        keep += [L, A, Rr]
        e.L, e.A, e.R = L.data_ptr(), A.data_ptr(), Rr.data_ptr()
        e.s, e.S = A.shape[0], A.shape[3]
        e.a_strides[:] = tuple(A.stride())
    rhs, inv_I = D.contig(rhs), D.contig(inv_I)
    sol = D.empty(*xs)
    rc = ctypes.c_double(0.0)
    D._stream()
    st = lib.ttk_dense_schur_solve(D.ctx(), r, n, R, arr, rhs.data_ptr(), inv_I.data_ptr(), sol.data_ptr(),
                                   ctypes.byref(rc))
    if st == _TTK_ILL_CONDITIONED:
        raise D.LinAlgWarning(f"Ill-conditioned matrix (rcond={rc.value:.5g}): result may not be accurate.")
    D.check(st, "dense_schur_solve")
    return sol


def _fbsub_(LZ, B):
    """forward_backward_sub (`src/tt_ipm.py:178-181`) in place on B (n, k)."""
    D.trsm_(LZ, B, trans=False)
    D.trsm_(LZ, B, trans=True)
    return B


_LOCAL_TRACE = bool(os.environ.get("TTIPM_LOCAL_TRACE"))  # diagnostics: one line per local KKT solve


def _run_lgmres(op, rhs_flat, m, rtol):
    restart = min(m, 100)
    aug = max(restart // 10, 3)
    info = {}
    x = lgmres(op.matvec_into, rhs_flat, rtol=rtol, max_it=300, restart=restart, augment=aug,
               native=getattr(op, "h", 0), info=info)
    if D.ALGO is not None:  # applications made inside native chunks (the others counted themselves)
        D.count_algo(info.get("native_matvecs", 0) * op.mv_flops(), info.get("native_matvecs", 0), "schur_matvec")
    if _LOCAL_TRACE:
        print(f"  lgmres n={rhs_flat.numel()} restart={restart} its={info.get('its')} matvecs={info.get('matvecs')} "
              f"reason={info.get('reason')}")
    return x


def _dense_python(XAX_k, A_k, XAX_k1, rhs, inv_I, xs):
    """The dense branch of `_ipm_local_solver` (`src/tt_ipm.py:200-222`) step by step."""
    r, n, R = xs[0], xs[2], xs[3]
    m = r * n * R
    rd = D.clone(rhs[:, 1]).view(m, 1)
    rc = D.clone(rhs[:, 2]).view(m, 1)
    rp = D.clone(rhs[:, 0]).view(m, 1)
    LXI = _assemble(XAX_k, A_k, XAX_k1, (2, 2), m)
    D.mul_(LXI, LXI, inv_I.view(1, m).expand(m, m))
    Leq = _assemble(XAX_k, A_k, XAX_k1, (0, 1), m)
    LZ = _assemble(XAX_k, A_k, XAX_k1, (2, 1), m)
    D.cholesky_(LZ)
    t = D.clone(rc)
    D.matmul(LXI, rd, out=t, alpha=-1.0, beta=1.0)
    _fbsub_(LZ, t)
    bvec = D.clone(rp)
    D.matmul(Leq, t, out=bvec, alpha=-1.0, beta=1.0)
    _fbsub_(LZ, LXI)
    T1 = D.matmul(LXI, Leq.t())
    Am = D.matmul(Leq, T1)
    einsum(ASSEMBLE, XAX_k[0, 0], A_k[0, 0], XAX_k1[0, 0], out=Am.view(r, n, R, r, n, R), beta=1.0)
    D.add_diag_(Am, 1e-11)
    piv = D.lu_(Am)
    D.lu_solve_(Am, piv, bvec)
    sol = D.empty(*xs)
    D.copy_(sol[:, 0], bvec.view(r, n, R))
    t2 = D.clone(rd).view(r, n, R)
    einsum(APPLY_T, XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], sol[:, 0], out=t2, alpha=-1.0, beta=1.0)
    D.mul_(sol[:, 2], t2, inv_I)
    t3 = D.clone(rc).view(r, n, R)
    einsum(APPLY, XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], sol[:, 2], out=t3, alpha=-1.0, beta=1.0)
    _fbsub_(LZ, t3.view(m, 1))
    D.copy_(sol[:, 1], t3)
    return sol


def _lgmres_prologue(XAX_k, A_k, XAX_k1, inv_I, rhs, prev, xs, nb2):
    """the Schur operator, the reduced right-hand side and its residual at `prev` (the iterative
    branch of `src/tt_ipm.py:224-262`); <lrhs, lrhs> and ||lrhs - S prev||^2 into the device slots
    nb2[0:2] (unread)."""
    r, n, R = xs[0], xs[2], xs[3]
    m = r * n * R
    op = MatVecWrapper(XAX_k, A_k, XAX_k1, inv_I, (r, n, R))
    lrhs = D.empty(2 * m)
    l0, l1 = lrhs[:m].view(r, n, R), lrhs[m:].view(r, n, R)
    D.copy_(l0, rhs[:, 0])
    D.copy_(l1, rhs[:, 2])
    w = D.empty(r, n, R)
    D.mul_(w, inv_I, rhs[:, 1])
    einsum(APPLY, XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], w, out=l1, alpha=-1.0, beta=1.0)
    D.dot_into(lrhs, lrhs, nb2[0:1])
    pv = D.empty(2 * m)
    D.copy_(pv.view(2, r, n, R), prev[:, :2].permute(1, 0, 2, 3))
    lvec = op.matvec(pv)
    diff = D.clone(lrhs)
    D.copy_(diff, lvec, -1.0, 1.0)
    D.dot_into(diff, diff, nb2[1:2])
    return op, lrhs, diff


def _ipm_local_solver(XAX_k, A_k, XAX_k1, Xb_k, b_k, Xb_k1, prev, size_limit, dense_solve=True, rtol=1e-5,
                      res_out=None):
    """`_ipm_local_solver` (`src/tt_ipm.py:183-282`) on the device.

    Host waits: when the dense branch is ruled out by size or by the caller, the iterative branch's
    prologue is enqueued before ANY read and its two norms come back with ||rhs|| and the old
    residual in one read.  `res_out` (a device slot): the new residual's square is left there unread
    and the returned res_new is None -- the caller reads it with its next device scalars and applies
    `if res_old < res_new: sol = prev` itself (`_finish_local`)."""
    xs = tuple(prev.shape)
    r, n, R = xs[0], xs[2], xs[3]
    m = r * n * R
    rhs = _local_rhs(Xb_k, b_k, Xb_k1, xs, 3)
    inv_I = D.recip(einsum(DIAG, XAX_k[1, 2], A_k[1, 2], XAX_k1[1, 2]))
    pro, nv = None, None
    if (np.sqrt(r * R) <= size_limit) and dense_solve:
        nrhs, res_old = _rhs_and_residual_norms(A_k, XAX_k, XAX_k1, prev, rhs)
    else:  # iterative branch whatever res_old is: one read for all four dots
        buf = D.empty(4)
        _rhs_and_residual_dots(A_k, XAX_k, XAX_k1, prev, rhs, buf[0:2])
        pro = _lgmres_prologue(XAX_k, A_k, XAX_k1, inv_I, rhs, prev, xs, buf[2:4])
        h = D.read(buf)
        nrhs, res_old = _norms_from_dots(h[0:2])
        nv = h[2:4]
    dense_solve = (np.sqrt(r * R) <= size_limit) and dense_solve and (res_old >= rtol)
    failed = not dense_solve
    sol = None
    if dense_solve:
        try:
            dense = _dense_native if NATIVE_DENSE and D.DEV.type == "cuda" else _dense_python
            sol = dense(XAX_k, A_k, XAX_k1, rhs, inv_I, xs)
        except Exception as e:
            print(e)
            _report(e)
            failed = True
    if not dense_solve or failed:
        if pro is None:
            nb2 = D.empty(2)
            pro = _lgmres_prologue(XAX_k, A_k, XAX_k1, inv_I, rhs, prev, xs, nb2)
            nv = D.read(nb2)
        op, lrhs, diff = pro
        lnorm = D.norm_of(nv[0])
        use_prev = D.norm_of(nv[1]) < lnorm
        if use_prev:
            lrhs = diff
        it_fail = False
        try:
            lsol = _run_lgmres(op, lrhs, m, rtol)
        except Exception as e:
            _report(e)
            it_fail = True
            failed = True
            sol = prev
        if not it_fail:
            sol = D.empty(*xs)
            D.copy_(sol[:, :2], lsol.view(2, r, n, R).permute(1, 0, 2, 3))
            if use_prev:
                D.copy_(sol[:, :2], prev[:, :2], 1.0, 1.0)
            zt = D.clone(rhs[:, 1])
            einsum(APPLY_T, XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], sol[:, 0], out=zt, alpha=-1.0, beta=1.0)
            D.mul_(sol[:, 2], inv_I, zt)
    if res_out is not None:
        _residual_norm(A_k, XAX_k, XAX_k1, sol, rhs, nrhs, res_out)
        return sol, res_old, None, rhs, nrhs, failed
    res_new = _residual_norm(A_k, XAX_k, XAX_k1, sol, rhs, nrhs)
    if _LOCAL_TRACE:
        print(f"  local m={m} dense={dense_solve} failed={failed} res_old={res_old:.6e} res_new={res_new:.6e}")
    if res_old < res_new:
        sol = prev
    return sol, res_old, min(res_old, res_new), rhs, nrhs, failed


def _dense_python_ineq(XAX_k, A_k, XAX_k1, rhs, inv_I, xs):
    """The dense branch of `_ipm_local_solver_ineq` (`src/tt_ipm.py:303-352`) step by step."""
    r, n, R = xs[0], xs[2], xs[3]
    m = r * n * R
    LZ = _assemble(XAX_k, A_k, XAX_k1, (2, 1), m)
    D.cholesky_(LZ)
    rp, rd, rc, rt = (D.clone(rhs[:, i]).view(m, 1) for i in range(4))
    LZ_rc = _fbsub_(LZ, D.clone(rc))
    LZ_LX = _fbsub_(LZ, _assemble(XAX_k, A_k, XAX_k1, (2, 2), m))
    Leq = _assemble(XAX_k, A_k, XAX_k1, (0, 1), m)
    Top = _assemble(XAX_k, A_k, XAX_k1, (3, 1), m)
    LZ_LXI = D.empty(m, m)
    D.mul_(LZ_LXI, LZ_LX, inv_I.view(1, m).expand(m, m))
    w = D.clone(LZ_rc)
    D.matmul(LZ_LXI, rd, out=w, alpha=-1.0, beta=1.0)
    u = D.clone(rp)
    D.matmul(Leq, w, out=u, alpha=-1.0, beta=1.0)
    v = D.clone(rt)
    D.matmul(Top, w, out=v, alpha=-1.0, beta=1.0)
    Am = _assemble(XAX_k, A_k, XAX_k1, (0, 0), m)
    D.matmul(Leq, D.matmul(LZ_LXI, Leq.t()), out=Am, beta=1.0)
    Dm = _assemble(XAX_k, A_k, XAX_k1, (3, 3), m)
    D.matmul(Top, LZ_LX, out=Dm, beta=1.0)
    D.add_diag_(Dm, 1e-11)
    Top2 = D.matmul(D.matmul(Top, LZ_LXI), Leq.t())
    Leq2 = D.matmul(Leq, LZ_LX)
    dpiv = D.lu_(Dm, check_rcond=False)
    Dv = D.clone(v)
    D.lu_solve_(Dm, dpiv, Dv)
    D.matmul(Leq2, Dv, out=u, alpha=-1.0, beta=1.0)
    DT = D.clone(Top2)
    D.lu_solve_(Dm, dpiv, DT)
    D.matmul(Leq2, DT, out=Am, alpha=-1.0, beta=1.0)
    piv = D.lu_(Am, check_rcond=False)
    y = D.clone(u)
    D.lu_solve_(Am, piv, y)
    sol = D.empty(*xs)
    D.copy_(sol[:, 0], y.view(r, n, R))
    D.matmul(Top2, y, out=v, alpha=-1.0, beta=1.0)
    D.lu_solve_(Dm, dpiv, v)
    D.copy_(sol[:, 3], v.view(r, n, R))
    t2 = D.clone(rd).view(r, n, R)
    einsum(APPLY_T, XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], sol[:, 0], out=t2, alpha=-1.0, beta=1.0)
    D.mul_(sol[:, 2], t2, inv_I)
    D.copy_(sol[:, 2], sol[:, 3], -1.0, 1.0)
    t3 = D.clone(rc).view(r, n, R)
    einsum(APPLY, XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], sol[:, 2], out=t3, alpha=-1.0, beta=1.0)
    _fbsub_(LZ, t3.view(m, 1))
    D.copy_(sol[:, 1], t3)
    return sol


def _dense_native_ineq(XAX_k, A_k, XAX_k1, rhs, inv_I, xs):
    """`ttk_dense_schur_solve_ineq`: the dense branch of `_ipm_local_solver_ineq` in one library call
    (NOT_PD / SINGULAR raise LinAlgError like the Python steps' Cholesky / LU)."""
    r, n, R = xs[0], xs[2], xs[3]
    keys = ((0, 0), (0, 1), (2, 1), (2, 2), (3, 1), (3, 3))
    arr = (_LocalBlock * len(keys))()
    keep = []
    for e, key in zip(arr, keys):
        L, A, Rr = D.contig(XAX_k[key]), A_k[key], D.contig(XAX_k1[key])
        keep += [L, A, Rr]
        e.L, e.A, e.R = L.data_ptr(), A.data_ptr(), Rr.data_ptr()
        e.s, e.S = A.shape[0], A.shape[3]
        e.a_strides[:] = tuple(A.stride())
    rhs, inv_I = D.contig(rhs), D.contig(inv_I)
    sol = D.empty(*xs)
    D._stream()
    D.check(lib.ttk_dense_schur_solve_ineq(D.ctx(), r, n, R, arr, rhs.data_ptr(), inv_I.data_ptr(), sol.data_ptr()),
            "dense_schur_solve_ineq")
    return sol


def _ipm_local_solver_ineq(XAX_k, A_k, XAX_k1, Xb_k, b_k, Xb_k1, prev, size_limit, dense_solve=True, rtol=1e-5,
                           res_out=None):
    """`_ipm_local_solver_ineq` (`src/tt_ipm.py:284-401`) on the device (`res_out` as in
    `_ipm_local_solver`)."""
    xs = tuple(prev.shape)
    r, n, R = xs[0], xs[2], xs[3]
    m = r * n * R
    rhs = _local_rhs(Xb_k, b_k, Xb_k1, xs, 4)
    inv_I = D.recip(einsum(DIAG, XAX_k[1, 2], A_k[1, 2], XAX_k1[1, 2]))
    nrhs, res_old = _rhs_and_residual_norms(A_k, XAX_k, XAX_k1, prev, rhs)
    dense_solve = (np.sqrt(r * R) <= 0.95 * size_limit) and dense_solve and (res_old >= rtol)
    failed = not dense_solve
    sol = None
    if dense_solve:
        try:
            dense = _dense_native_ineq if NATIVE_DENSE and D.DEV.type == "cuda" else _dense_python_ineq
            sol = dense(XAX_k, A_k, XAX_k1, rhs, inv_I, xs)
        except Exception as e:
            _report(e)
            failed = True
    if not dense_solve or failed:
        op = IneqMatVecWrapper(XAX_k, A_k, XAX_k1, inv_I, (r, n, R))
        lrhs = D.empty(3 * m)
        l0, l1, l2 = (lrhs[i * m:(i + 1) * m].view(r, n, R) for i in range(3))
        D.copy_(l0, rhs[:, 0])
        D.copy_(l1, rhs[:, 2])
        w = D.empty(r, n, R)
        D.mul_(w, inv_I, rhs[:, 1])
        einsum(APPLY, XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], w, out=l1, alpha=-1.0, beta=1.0)
        D.copy_(l2, rhs[:, 3])
        lnorm = D.norm(lrhs)
        pv = D.empty(3 * m)
        pv3 = pv.view(3, r, n, R)
        D.copy_(pv3[0], prev[:, 0])
        D.copy_(pv3[1], prev[:, 1])
        D.copy_(pv3[2], prev[:, 3])
        lvec = op.matvec(pv)  # raises like the reference when INEQ_MATVEC_BUG (outside any try)
        diff = D.clone(lrhs)
        D.copy_(diff, lvec, -1.0, 1.0)
        use_prev = D.norm(diff) < lnorm
        if use_prev:
            lrhs = diff
        it_fail = False
        try:
            lsol = _run_lgmres(op, lrhs, m, rtol)
        except Exception as e:
            _report(e)
            it_fail = True
            failed = True
            sol = prev
        if not it_fail:
            l3 = lsol.view(3, r, n, R)
            if use_prev:
                D.copy_(l3[0], prev[:, 0], 1.0, 1.0)
                D.copy_(l3[1], prev[:, 1], 1.0, 1.0)
                D.copy_(l3[2], prev[:, 3], 1.0, 1.0)
            zt = D.clone(rhs[:, 1])
            einsum(APPLY_T, XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], l3[0], out=zt, alpha=-1.0, beta=1.0)
            sol = D.empty(*xs)
            D.mul_(sol[:, 2], inv_I, zt)
            D.copy_(sol[:, 2], l3[2], -1.0, 1.0)
            D.copy_(sol[:, 0], l3[0])
            D.copy_(sol[:, 1], l3[1])
            D.copy_(sol[:, 3], l3[2])
    if res_out is not None:
        _residual_norm(A_k, XAX_k, XAX_k1, sol, rhs, nrhs, res_out)
        return sol, res_old, None, rhs, nrhs, failed
    res_new = _residual_norm(A_k, XAX_k, XAX_k1, sol, rhs, nrhs)
    if res_old < res_new:
        sol = prev
    return sol, res_old, min(res_old, res_new), rhs, nrhs, failed


# ------------------------------------------------------------------ IPM driver (`:404-1099`)
class IneqStatus(Enum):
    ACTIVE = 0
    SETTING_ACTIVE = 1
    SETTING_INACTIVE = 2
    INACTIVE = 3
    NOT_IN_USE = 4

    def __str__(self):
        return self.name.lower().replace('_', ' ')


@dataclass
class IPMStatus:
    dim: int
    feasibility_tol: float
    centrality_tol: float
    op_tol: float
    eps: float
    aho_direction: bool
    is_primal_feasible: bool
    primal_error: float
    is_dual_feasible: bool
    dual_error: float
    is_central: bool
    centrality_error: float
    mu: float
    is_last_iter: bool
    ineq_status: IneqStatus
    verbose: bool
    primal_error_normalisation: float
    dual_error_normalisation: float
    mals_rank_restriction: int
    boundary_val: float = 1e-10
    ineq_boundary_val: float = 0.01
    sigma: float = 0.5
    num_ineq_constraints: float = 0
    lag_map_t = None
    lag_map_y = None
    compl_ineq_mask = None
    mals_delta0 = None
    eigen_x0 = None
    eigen_z0 = None
    eigen_xt0 = None
    eigen_zt0 = None
    kkt_iterations = 7
    centrl_error_normalisation: float = 1.0
    eta = 1e-3


def tt_compute_primal_feasibility(L, b, X, st):
    """`src/tt_ipm.py:404-407`"""
    e = 0.01 * st.eta * st.primal_error_normalisation
    return T.tt_rank_reduce(T.tt_sub(tt_mat_vec_mul(L, T.tt_reshape(X, (4,)), e, st.eps), b), e)


def tt_compute_dual_feasibility(C, Ladj, Z, Y, Tt, st):
    """`src/tt_ipm.py:410-417`"""
    act = st.ineq_status is IneqStatus.ACTIVE
    df = T.tt_rank_reduce(T.tt_sub(T.tt_fast_matrix_vec_mul(Ladj, Y, st.eps),
                                   T.tt_rank_reduce(T.tt_add(T.tt_reshape(Z, (4,)), C), st.eps)),
                          st.eps if act else 0.01 * st.eta * st.dual_error_normalisation)
    if act and Tt is not None:
        df = T.tt_rank_reduce(T.tt_sub(df, T.tt_reshape(Tt, (4,))), 0.01 * st.eta * st.dual_error_normalisation)
    return df


def tt_compute_centrality(X, Z, st):
    """`src/tt_ipm.py:420-426`"""
    e = 0.01 * st.eta * st.centrl_error_normalisation
    if st.aho_direction:
        return T.tt_reshape(T.tt_scale(-1, _tt_symmetrise(tt_mat_mat_mul(X, Z, e, st.eps), e)), (4,))
    return T.tt_reshape(T.tt_scale(-1, tt_mat_mat_mul(Z, X, e, st.eps)), (4,))


def tt_infeasible_newton_system(lhs, C, X, Y, Z, Tt, L, Ladj, b, mask, st):
    """`src/tt_ipm.py:429-475`"""
    rhs = TTBlockVector()
    # the residual norms are read once, after every device step that does not depend on them (the
    # same steps in the same order: the random core picks of tt_scale stay where they were); the
    # centrality row is built there too when it is certain to be (not central), and its norm -- the
    # KKT row scaling's (`_tt_kkt_row_scales`) -- comes back in the same read
    pf = tt_compute_primal_feasibility(L, b, X, st)
    df = tt_compute_dual_feasibility(C, Ladj, Z, Y, Tt, st)
    if st.aho_direction:
        lhs[2, 1] = T.tt_psd_rank_reduce(T.tt_scale(0.5, T.tt_add(T.tt_IkronM(Z), T.tt_MkronI(Z))),
                                         eps=0.1 * st.eta * st.dual_error_normalisation)
        lhs[2, 2] = T.tt_psd_rank_reduce(T.tt_scale(0.5, T.tt_add(T.tt_MkronI(X), T.tt_IkronM(X))),
                                         eps=0.1 * st.eta * st.primal_error_normalisation)
    else:
        lhs[2, 1] = T.tt_psd_rank_reduce(T.tt_MkronI(Z), eps=0.1 * st.eta * st.dual_error_normalisation)
        lhs[2, 2] = T.tt_psd_rank_reduce(T.tt_IkronM(X), eps=0.1 * st.eta * st.primal_error_normalisation)
    cen = None if st.is_central else tt_compute_centrality(X, Z, st)
    ips = T.tt_scalars([("ip", pf, pf), ("ip", df, df)] + ([("ip", cen, cen)] if cen is not None else []))
    npf, ndf = T.norm_from_ip(ips[0]), T.norm_from_ip(ips[1])
    st.primal_error = np.divide(npf, st.primal_error_normalisation)
    st.is_primal_feasible = np.less(st.primal_error, st.feasibility_tol)
    st.dual_error = np.divide(ndf, st.dual_error_normalisation)
    st.is_dual_feasible = np.less(st.dual_error, (1 + (st.ineq_status is IneqStatus.ACTIVE)) * st.feasibility_tol)
    st.is_last_iter = st.is_last_iter or (st.is_primal_feasible and st.is_dual_feasible and st.is_central)
    # the row norms the KKT row scaling reads (`_tt_kkt_row_scales`) are these same values: kept with
    # the row objects instead of being recomputed
    rhs._norms = {}
    if not st.is_primal_feasible or st.is_last_iter:
        rhs[0] = pf
        rhs._norms[0] = (pf, npf)
    if not st.is_dual_feasible or st.is_last_iter:
        rhs[1] = df
        rhs._norms[1] = (df, ndf)
    if cen is not None:
        rhs[2] = cen
        rhs._norms[2] = (cen, T.norm_from_ip(ips[2]))
    elif st.is_last_iter:
        rhs[2] = tt_compute_centrality(X, Z, st)
    if st.ineq_status is IneqStatus.ACTIVE:
        lhs[3, 1] = T.tt_diag_op(Tt, 0.1 * st.eta * st.dual_error_normalisation)
        mX = T.tt_rank_reduce(T.tt_add(T.tt_scale(st.ineq_boundary_val, mask), T.tt_fast_hadamard(mask, X, st.eps)),
                              eps=st.eps)
        lhs[3, 3] = T.tt_rank_reduce(T.tt_add(st.lag_map_t, T.tt_diag_op(mX, st.eps)),
                                     eps=0.1 * st.eta * st.dual_error_normalisation)
        if not st.is_central or st.is_last_iter:
            rhs[3] = T.tt_rank_reduce(T.tt_reshape(T.tt_scale(-1, T.tt_fast_hadamard(mX, Tt, st.eps)), (4,)),
                                      eps=0.01 * st.eta * st.centrl_error_normalisation)
    return lhs, rhs, st


def _tt_symmetrise(M, e):
    return T.tt_rank_reduce(T.tt_scale(0.5, T.tt_add(M, T.tt_transpose(M))), eps=e)


def _tt_psd_symmetrise(M, e):
    return T.tt_psd_rank_reduce(T.tt_scale(0.5, T.tt_add(M, T.tt_transpose(M))), eps=e)


def _tt_mask_symmetrise(M, mask, e):
    return T.tt_mask_rank_reduce(T.tt_scale(0.5, T.tt_add(M, T.tt_transpose(M))), mask, eps=e)


def _tt_copy(tt):
    return D.clone_many(tt)


def _tt_scale_nondestructive(tt, s):
    if tt is None or np.isclose(s, 1.0):
        return tt
    return T.tt_scale(s, _tt_copy(tt))


def _tt_rhs_row_norm(rhs, i):
    row = rhs.get_row(i)
    if row is None:
        return 0.0
    cached = getattr(rhs, "_norms", {}).get(i)
    n = cached[1] if cached is not None and cached[0] is row else T.tt_norm(row)
    return float(n) if np.isfinite(n) else 0.0


def _tt_kkt_row_scales(rhs, st):
    """`src/tt_ipm.py:510-528`"""
    eps = max(st.op_tol, 1e-12)
    fn = max(_tt_rhs_row_norm(rhs, 0), _tt_rhs_row_norm(rhs, 1))
    cn = max(_tt_rhs_row_norm(rhs, 2), _tt_rhs_row_norm(rhs, 3))
    sc = {}
    if fn > eps:
        fs = float(np.clip(1.0 / max(fn, eps), 1e-6, 1e6))
        sc[0] = fs
        sc[1] = fs
    if cn > eps:
        cs = float(np.clip(1.0 / max(cn, eps), 1e-6, 1e6))
        if 0 in sc:
            cs = min(cs, sc[0])
        sc[2] = cs
        sc[3] = cs
    return sc


def _tt_effective_row_scale(lhs, key, sc):
    s = sc.get(key[0], 1.0)
    if key in lhs._transposes:
        cr, _ = lhs._transposes[key]
        if cr in sc:
            s = np.sqrt(s * sc[cr])
    if key in lhs._aliases:
        cr, _ = lhs._aliases[key]
        if cr in sc:
            s = np.sqrt(s * sc[cr])
    return float(s)


def _tt_build_row_scaled_kkt(lhs, rhs, st, row_scales=None):
    """`src/tt_ipm.py:545-568`"""
    sc = _tt_kkt_row_scales(rhs, st) if row_scales is None else row_scales
    if not sc:
        return lhs, rhs
    L = TTBlockMatrix()
    L._aliases = dict(lhs._aliases)
    L._transposes = dict(lhs._transposes)
    for key, blk in lhs._data.items():
        L[key] = _tt_scale_nondestructive(blk, _tt_effective_row_scale(lhs, key, sc))
    R = TTBlockVector()
    for i in rhs.keys():
        R[i] = _tt_scale_nondestructive(rhs.get_row(i), sc.get(i, 1.0))
    if st.verbose:
        print(f"KKT row scaling: feas={sc.get(0, sc.get(1, 1.0)):.2e}, cent={sc.get(2, sc.get(3, 1.0)):.2e}", flush=True)
    return L, R


def _ineq_step_size(Att, Dtt, e_tt, st):
    """`src/tt_ipm.py:730-747`"""
    s = T.tt_add(Att, Dtt)
    if st.compl_ineq_mask:
        s = T.tt_add(s, st.compl_ineq_mask)
    s = T.tt_rank_reduce(s, st.eps)
    e_tt, _ = tt_min_eig(T.tt_diag_op(s, st.eps), x0=e_tt, tol=1e-8, verbose=st.verbose)
    esq = T.tt_reshape(e_tt, (2, 2))
    if np.abs(T.tt_inner_prod(s, esq)) > st.eps:
        esq = T.tt_normalise(T.tt_fast_hadamard(esq, esq, st.eps))
        mA = np.abs(T.tt_inner_prod(Att, esq))
        mD = T.tt_inner_prod(Dtt, esq)
        step = 1 if mD >= -st.eps else np.clip(-mA / mD, a_min=0, a_max=1)
    else:
        step = 1
    return step, e_tt


def _tt_get_ineq_step_sizes(xs, zs, X, Tt, DX, DT, mask, st):
    """`src/tt_ipm.py:750-779`"""
    if xs > 0:
        mX = T.tt_fast_hadamard(mask, X, st.eps)
        mDX = T.tt_fast_hadamard(mask, DX, st.eps)
        xis, st.eigen_xt0 = _ineq_step_size(T.tt_add(mX, T.tt_scale(st.ineq_boundary_val, mask)),
                                            T.tt_scale(xs, mDX), st.eigen_xt0, st)
        if not st.is_last_iter:
            if 1 - xis < st.op_tol and T.tt_norm(Tt) < st.op_tol:
                if st.ineq_status is IneqStatus.ACTIVE:
                    st.ineq_status = IneqStatus.SETTING_INACTIVE
            else:
                if st.ineq_status is IneqStatus.INACTIVE:
                    st.ineq_status = IneqStatus.SETTING_ACTIVE
        xs *= xis
    if zs > 0 and st.ineq_status is IneqStatus.ACTIVE:
        ts, st.eigen_zt0 = _ineq_step_size(Tt, T.tt_scale(zs, DT), st.eigen_zt0, st)
        zs *= ts
    return xs, zs


_DUMP_DIR = os.environ.get("TTIPM_DUMP_STEP")  # diagnostics: dump step-size eigenproblem inputs
_dump_count = [0]


def _dump_step_inputs(X, Z, DX, DZ, x0s, rng, xs, zs):
    """Write the inputs/outputs of one `_tt_get_step_sizes` eigen pair to TTIPM_DUMP_STEP/step_NNN.npz
    (replayed against the oracle by tools/replay_step.py)."""
    arr = {"xs": xs, "zs": zs, "rng_key": rng[1], "rng_pos": rng[2], "rng_g": rng[3], "rng_c": rng[4]}
    for name, tt in (("X", X), ("Z", Z), ("DX", DX), ("DZ", DZ), ("x0", x0s[0]), ("z0", x0s[1])):
        if tt is None:
            continue
        arr[name + "/n"] = len(tt)
        for i, c in enumerate(tt):
            arr[f"{name}/{i}"] = D.read(c)
    os.makedirs(_DUMP_DIR, exist_ok=True)
    np.savez(os.path.join(_DUMP_DIR, f"step_{_dump_count[0]:03d}.npz"), **arr)
    _dump_count[0] += 1


def _tt_get_step_sizes(X, Z, Tt, DX, DZ, DT, mask, st):
    """`src/tt_ipm.py:700-727`"""
    if st.is_last_iter:
        X = T.tt_add(X, T.tt_scale(st.boundary_val, T.tt_identity(len(X))))
        Z = T.tt_add(Z, T.tt_scale(st.boundary_val, T.tt_identity(len(Z))))
    x0s = (st.eigen_x0, st.eigen_z0)
    rng = _rng.R().get_state()
    xs, st.eigen_x0 = tt_max_generalised_eigen(X, DX, x0=st.eigen_x0, tol=1e-8, verbose=st.verbose)
    zs, st.eigen_z0 = tt_max_generalised_eigen(Z, DZ, x0=st.eigen_z0, tol=1e-8, verbose=st.verbose)
    if _DUMP_DIR:
        _dump_step_inputs(X, Z, DX, DZ, x0s, rng, xs, zs)
    if st.ineq_status is not IneqStatus.NOT_IN_USE:
        if st.is_last_iter:
            X = T.tt_add(X, T.tt_scale(st.ineq_boundary_val + st.boundary_val, mask))
            Tt = T.tt_add(Tt, T.tt_scale(st.ineq_boundary_val + st.boundary_val, mask))
        xs, zs = _tt_get_ineq_step_sizes(xs, zs, X, Tt, DX, DT, mask, st)
    tau = 0.9 + 0.05 * min(xs, zs)
    if st.verbose:
        print("Step search concluded.")
        print(f"Step sizes: a_p:{xs:.2e}, a_d:{zs:.2e}", flush=True)
    return tau * xs, tau * zs


def _tt_ipm_newton_step(lhs, rhs, mask, X, Z, Tt, ZX, TX, st, solver):
    """`_tt_ipm_newton_step` (`src/tt_ipm.py:571-697`)."""
    try:
        if st.verbose:
            print("\n--- Predictor  step ---", flush=True)
        sc = _tt_kkt_row_scales(rhs, st)
        Lp, Rp = _tt_build_row_scaled_kkt(lhs, rhs, st, sc)
        Dl, _ = solver(Lp, Rp, st.mals_delta0, st.kkt_iterations + st.is_last_iter, st.mals_rank_restriction, st.eta)
        st.mals_delta0 = Dl
        DX = _tt_symmetrise(T.tt_reshape(_tt_get_block(1, Dl), (2, 2)), st.eps)
        DZ = _tt_symmetrise(T.tt_reshape(_tt_get_block(2, Dl), (2, 2)), st.eps)
        DY = T.tt_rank_reduce(_tt_get_block(0, Dl), eps=st.eps)
        DT = None
        if st.ineq_status is IneqStatus.ACTIVE:
            DT = T.tt_rank_reduce(_tt_get_block(3, Dl), eps=st.eps)
            DT = T.tt_fast_hadamard(mask, T.tt_reshape(DT, (2, 2)), st.eps)
        xs, zs = _tt_get_step_sizes(X, Z, Tt, DX, DZ, DT, mask, st)
        if not st.is_central and not st.is_last_iter:
            act = st.ineq_status is IneqStatus.ACTIVE
            sv = T.tt_scalars([("ip", DX, DZ), ("ip", X, DZ), ("ip", DX, Z)]
                              + ([("ip", DT, DX), ("ip", X, DT), ("sum", DT), ("ip", DX, Tt)] if act else []))
            DXZ = sv[0]
            if st.verbose:
                print("\n--- Centering-Corrector  step ---", flush=True)
            if act:
                mu_aff = (ZX + xs * zs * DXZ + zs * sv[1] + xs * sv[2]
                          + TX + xs * zs * sv[3]
                          + zs * (sv[4] + st.ineq_boundary_val * sv[5])
                          + xs * sv[6])
                e = max(1, 3 * min(xs, zs) ** 2)
                st.sigma = min(0.99, max(mu_aff / (ZX + TX), 0) ** e)
                if st.sigma > 1e-4:
                    rhs[3] = T.tt_rank_reduce(T.tt_add(T.tt_scale(st.sigma * st.mu, T.tt_reshape(mask, (4,))),
                                                       rhs.get_row(3)), 0.1 * st.eta * st.centrl_error_normalisation)
            else:
                mu_aff = ZX + xs * zs * DXZ + zs * sv[1] + xs * sv[2]
                e = max(1, 3 * min(xs, zs) ** 2)
                st.sigma = min(0.99, max(mu_aff / ZX, 0) ** e)
            ce = 0.1 * st.eta * st.centrl_error_normalisation
            if DXZ > 0.1 * st.centrality_tol:
                term = tt_compute_centrality(DX, DZ, st)
                if st.sigma > 1e-4:
                    rhs[2] = T.tt_rank_reduce(T.tt_add(T.tt_scale(st.sigma * st.mu, T.tt_reshape(T.tt_identity(len(X)), (4,))),
                                                       T.tt_add(rhs.get_row(2), term)), ce)
                else:
                    rhs[2] = T.tt_rank_reduce(T.tt_add(rhs.get_row(2), term), ce)
            else:
                if st.sigma > 1e-4:
                    rhs[2] = T.tt_rank_reduce(T.tt_add(T.tt_scale(st.sigma * st.mu, T.tt_reshape(T.tt_identity(len(X)), (4,))),
                                                       rhs.get_row(2)), ce)
                else:
                    rhs[2] = rhs.get_row(2)
            Lc, Rc = _tt_build_row_scaled_kkt(lhs, rhs, st, sc)
            Dc, _ = solver(Lc, Rc, st.mals_delta0, st.kkt_iterations + st.is_last_iter, st.mals_rank_restriction, st.eta)
            st.mals_delta0 = Dc
            DXc = _tt_symmetrise(T.tt_reshape(_tt_get_block(1, Dc), (2, 2)), st.eps)
            DZc = _tt_symmetrise(T.tt_reshape(_tt_get_block(2, Dc), (2, 2)), st.eps)
            DYc = T.tt_rank_reduce(_tt_get_block(0, Dc), eps=st.eps)
            DX = T.tt_rank_reduce(T.tt_add(DXc, DX), eps=st.eps)
            DY = T.tt_rank_reduce(T.tt_add(DYc, DY), eps=st.eps)
            DZ = T.tt_rank_reduce(T.tt_add(DZc, DZ), eps=st.eps)
            if st.ineq_status is IneqStatus.ACTIVE:
                DTc = T.tt_rank_reduce(_tt_get_block(3, Dc), eps=st.eps)
                DTc = T.tt_fast_hadamard(mask, T.tt_reshape(DTc, (2, 2)), st.eps)
                DT = T.tt_rank_reduce(T.tt_add(DTc, DT), eps=st.eps)
            xs, zs = _tt_get_step_sizes(X, Z, Tt, DX, DZ, DT, mask, st)
        else:
            st.sigma = 0
    except Exception as e:
        print(f"\n\t⚠️ Attention: {e}")
        print("\n\t==> Full traceback (most recent call last):")
        traceback.print_exc(file=sys.stdout)
        return 0, 0, None, None, None, None, st
    return xs, zs, DX, DY, DZ, DT, st


def _initialise(mask, st, dim, lam, lam_ineq):
    """`src/tt_ipm.py:782-794`"""
    X = T.tt_scale(lam, T.tt_identity(dim))
    Z = T.tt_scale(lam, T.tt_identity(dim))
    Y = T.tt_reshape(T.tt_zero_matrix(dim), (4,))
    Tt = None
    if st.ineq_status is IneqStatus.ACTIVE:
        Tt = T.tt_scale(lam_ineq, mask)
        xs, _ = tt_max_generalised_eigen(X, mask, tol=1e-7, verbose=st.verbose)
        X = T.tt_rank_reduce(T.tt_add(X, T.tt_scale(0.1 * xs, mask)), 0.1 * st.eta * st.primal_error_normalisation)
    return X, Y, Z, Tt


def _ipm_check_for_stalled_progress(prev, st, gap_tol):
    """`src/tt_ipm.py:853-866`"""
    if st.is_last_iter:
        return False
    if (abs(prev['primal'] - st.primal_error) < 0.04 * gap_tol and abs(prev['dual'] - st.dual_error) < 0.04 * gap_tol
            and abs(prev['centrality'] - st.centrality_error) < 0.02 * gap_tol):
        if st.verbose:
            print("============================================\n Progress stalled! Entering finishing phase.\n"
                  "============================================")
        return True
    return False


def _ipm_check_convergence(st, fin, ZX, TX, abs_tol, max_ref):
    """`src/tt_ipm.py:869-888`"""
    if not st.is_last_iter:
        return st, fin
    if abs(ZX) + abs(TX) < abs_tol and st.primal_error < abs_tol and st.dual_error < abs_tol:
        if st.verbose:
            print("Absolute tolerance reached!")
        fin = 0
    else:
        fin -= 1
        st.boundary_val = 0.001 * (1 - (fin / max_ref))
        if fin == 1:
            st.kkt_iterations += 1
    return st, fin


def _ipm_log_iteration(it, st, X, Y, Z, Tt):
    """`src/tt_ipm.py:891-898`"""
    print(f"\n--- Iteration {it - 1} ---")
    print(f"Status: Finishing up={st.is_last_iter}, Ineq={str(st.ineq_status)}")
    print(f"Feasibility: Central={st.is_central}, Primal={st.is_primal_feasible}, Dual={st.is_dual_feasible}")
    print(f"Direction: {'AHO' if st.aho_direction else 'XZ'}, Sigma: {st.sigma:.2e}")
    print(f"Errors: Centrality={st.centrality_error:.4e}, Primal={st.primal_error:.4e}, Dual={st.dual_error:.4e}")
    print(f"Ranks: X={T.tt_ranks(X)}, Z={T.tt_ranks(Z)}, Y={T.tt_ranks(Y)}, T={T.tt_ranks(Tt) if Tt else 'N/A'}",
          flush=True)


def tt_ipm(lag_maps, obj_tt, lin_op_tt, bias_tt, ineq_mask=None, max_iter=100, max_refinement=5, warm_up=3,
           gap_tol=1e-4, aho_direction=True, op_tol=1e-5, abs_tol=8e-4, eps=1e-12, mals_restarts=3, r_max=1000,
           lambdaStar=1, lambdaStarIneq=1, epsilonDash=None, epsilonDashineq=None, verbose=False, trace=None,
           iter_callback=None):
    """`tt_ipm` (`src/tt_ipm.py:901-1099`).  `trace` (list) collects one record per Newton-system
    assembly; `iter_callback(iteration)` is invoked after each completed IPM iteration (bench)."""
    C, L, b, mask = obj_tt, lin_op_tt, bias_tt, ineq_mask
    dim = len(C)
    st = IPMStatus(len(C), 2 * gap_tol, gap_tol / np.sqrt(dim), op_tol, eps, aho_direction, False, np.inf, False,
                   np.inf, False, np.inf, np.inf, False,
                   IneqStatus.NOT_IN_USE if mask is None else IneqStatus.ACTIVE, verbose, 1, 1, r_max)
    lag_maps = {k: T.tt_rank_reduce(v, eps=eps) for k, v in lag_maps.items()}
    C = T.tt_rank_reduce(C, eps=eps)
    L = T.tt_rank_reduce(L, eps=eps)
    b = T.tt_rank_reduce(b, eps=eps)
    st.primal_error_normalisation = 1 + T.tt_norm(b)
    st.dual_error_normalisation = 1 + T.tt_norm(C)
    skel = TTBlockMatrix()
    skel[1, 2] = T.tt_reshape(T.tt_identity(2 * dim), (4, 4))

    def make_solver(ls):
        return lambda lhs, rhs, x0, nswp, restr, tol: tt_restarted_block_amen(
            lhs, rhs, rank_restriction=restr, x0=x0, local_solver=ls, op_tol=op_tol, termination_tol=tol,
            num_restarts=mals_restarts, inner_m=nswp, verbose=verbose)

    solver_ineq = make_solver(_ipm_local_solver_ineq)
    solver_eq = make_solver(_ipm_local_solver)
    if st.ineq_status is IneqStatus.ACTIVE:
        solver = solver_ineq
        st.num_ineq_constraints = T.tt_inner_prod(mask, mask)
        st.compl_ineq_mask = T.tt_rank_reduce(T.tt_sub(T.tt_one_matrix(dim), mask), eps=eps)
        st.lag_map_t = lag_maps["t"]
        skel.add_alias((1, 2), (1, 3))
    else:
        solver = solver_eq
        st.num_ineq_constraints = 0
    Ladj = T.tt_transpose(L)
    skel[0, 1] = T.tt_scale(-1, L)
    skel.add_alias((0, 1), (1, 0), is_transpose=True)
    skel[0, 0] = lag_maps["y"]
    st.lag_map_y = lag_maps["y"]
    X, Y, Z, Tt = _initialise(mask, st, dim, lambdaStar, lambdaStarIneq)
    it = 0
    fin = max_refinement
    prev = {'primal': np.inf, 'dual': np.inf, 'centrality': np.inf}
    lhs = skel
    while fin > 0:
        it += 1
        st.aho_direction = (it > warm_up)
        if max_iter - max_refinement == it - 1 and not st.is_last_iter:
            print("============================================\n Maximum #iterations reached!\n"
                  "============================================")
            st.is_last_iter = True
        act = st.ineq_status is IneqStatus.ACTIVE
        sv = T.tt_scalars([("ip", Z, X), ("ip", C, T.tt_reshape(X, (4,)))]
                          + ([("ip", X, Tt), ("sum", Tt)] if act else []))  # one host read
        ZX = sv[0]
        TX = (sv[2] + st.ineq_boundary_val * sv[3]) if act else 0
        st.mu = np.divide(abs(ZX) + abs(TX), (2 ** dim + (st.ineq_status is IneqStatus.ACTIVE) * st.num_ineq_constraints))
        st.centrl_error_normalisation = 1 + abs(sv[1])
        st.centrality_error = st.mu / st.centrl_error_normalisation
        st.is_central = np.less(st.centrality_error, st.centrality_tol)
        st.eta = max(min(st.eta, 2 * st.mu), st.op_tol)
        lhs_m, rhs_v, st = tt_infeasible_newton_system(lhs, C, X, Y, Z, Tt, L, Ladj, b, mask, st)
        if trace is not None:
            trace.append({"iter": it, "mu": float(st.mu), "primal_error": float(st.primal_error),
                          "dual_error": float(st.dual_error), "centrality_error": float(st.centrality_error),
                          "sigma": float(st.sigma), "ranksX": T.tt_ranks(X), "ranksZ": T.tt_ranks(Z),
                          "ranksY": T.tt_ranks(Y), "is_last_iter": bool(st.is_last_iter),
                          "t": time.time()})
        if verbose:
            _ipm_log_iteration(it, st, X, Y, Z, Tt)
        st, fin = _ipm_check_convergence(st, fin, ZX, TX, abs_tol, max_refinement)
        if fin == 0:
            it -= 1
            break
        xs, zs, DX, DY, DZ, DT, st = _tt_ipm_newton_step(lhs_m, rhs_v, mask, X, Z, Tt, ZX, TX, st, solver)
        if (DX is None and DZ is None) or (xs < 1e-5 and zs < 1e-5):
            if st.is_last_iter:
                break
            print("============================================\n Hit PSD boundary! Entering finishing phase.\n"
                  "============================================")
            st.is_last_iter = True
        else:
            e_p = 0.1 * st.eta * st.primal_error_normalisation
            e_d = 0.1 * st.eta * st.dual_error_normalisation
            if fin <= 1:
                X = _tt_symmetrise(T.tt_add(X, T.tt_scale(xs, DX)), e_p)
            else:
                X = _tt_psd_symmetrise(T.tt_add(X, T.tt_scale(xs, DX)), e_p)
            if fin <= 1:
                Z = _tt_symmetrise(T.tt_add(Z, T.tt_scale(zs, DZ)), e_d)
            else:
                Z = _tt_psd_symmetrise(T.tt_add(Z, T.tt_scale(zs, DZ)), e_d)
            Y = T.tt_rank_reduce(T.tt_add(Y, T.tt_scale(zs, DY)), st.eps)
            Y = T.tt_reshape(_tt_symmetrise(T.tt_reshape(T.tt_sub(Y, T.tt_fast_matrix_vec_mul(st.lag_map_y, Y, st.eps)),
                                                         (2, 2)), e_d), (4,))
            if st.ineq_status is IneqStatus.ACTIVE:
                if fin <= 1:
                    Tt = _tt_symmetrise(T.tt_add(Tt, T.tt_scale(zs, DT)), e_d)
                else:
                    Tt = _tt_mask_symmetrise(T.tt_add(Tt, T.tt_scale(zs, DT)), mask, e_d)
            elif st.ineq_status is IneqStatus.SETTING_INACTIVE:
                solver = solver_eq
                lhs = skel.get_submatrix(2, 2)
                st.mals_delta0 = None
                st.ineq_status = IneqStatus.INACTIVE
            elif st.ineq_status is IneqStatus.SETTING_ACTIVE:
                solver = solver_ineq
                lhs = skel
                st.mals_delta0 = None
                st.ineq_status = IneqStatus.ACTIVE
        if _ipm_check_for_stalled_progress(prev, st, gap_tol):
            st.is_last_iter = True
        prev['primal'] = st.primal_error
        prev['dual'] = st.dual_error
        prev['centrality'] = st.centrality_error
        if iter_callback is not None:
            iter_callback(it)
    D.check_handoffs()  # a timed-out in-launch hand-off (stale data) invalidates the solve
    rX, rZ, rY = T.tt_ranks(X), T.tt_ranks(Z), T.tt_ranks(Y)
    rT = T.tt_ranks(Tt) if Tt else [0] * (st.dim - 1)
    print("---Terminated---")
    print(f"Converged in {it} iterations.")
    print(f"Ranks: X={rX}, Z={rZ}, Y={rY}, T={rT}")
    info = {"num_iters": it, "ranksX": rX, "ranksY": rY, "ranksZ": rZ, "ranksT": rT, "status": st}
    return X, Y, Tt, Z, info
