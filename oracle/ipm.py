"""CPU restatement of the reference's IPM layer (`src/tt_ipm.py`) -- TEST INFRASTRUCTURE.

Contains the local KKT solvers (dense Schur path + PETSc-LGMRES path on the Schur-reduced
matvec of `cy_src/lgmres_cy.pyx`), the Newton system, predictor-corrector step and the outer
loop.  Warnings are escalated to errors exactly as the reference does (`src/tt_ipm.py:16`)
inside `tt_ipm` only, so the dense->iterative fallback triggers on the same conditions
(`LinAlgWarning` from an ill-conditioned `solve`, `LinAlgError` from `cholesky`)."""
import sys
import traceback
import warnings
from dataclasses import dataclass
from enum import Enum

import numpy as np
import scipy.linalg as sla

from . import tt as T
from .als import BlockMatrix, BlockVector, get_block, mat_mat_mul, mat_vec_mul, restarted_block_amen
from .eig import max_generalised_eigen, min_eig
from .petsc_lgmres import lgmres
from .tt import einsum

APPLY = "lsr,smnS,LSR,rnR->lmL"
APPLY_T = "lsr,smnS,LSR,lmL->rnR"
ASSEMBLE = "lsr,smnS,LSR->lmLrnR"
DIAG = "lsr,smnS,LSR->lmL"
RHS = "br,bmB,BR->rmR"

# when True, the inequality matvec reproduces the shipped bug (`cy_src/lgmres_cy.pyx:510`)
INEQ_MATVEC_BUG = False


class IneqMatvecBug(TypeError):
    pass


def _apply(L, A, R, v):
    return einsum(APPLY, L, A, R, v)


def _apply_t(L, A, R, v):
    return einsum(APPLY_T, L, A, R, v)


def _chain_operands(L, A, R):
    """Pre-transposed operands of `MatVecWrapper.__init__` (`cy_src/lgmres_cy.pyx:233-270`)."""
    return (np.ascontiguousarray(L.transpose(0, 2, 1).reshape(L.shape[0], -1).T),
            np.ascontiguousarray(A.reshape(A.shape[0] * A.shape[1], A.shape[2] * A.shape[3]).T),
            np.ascontiguousarray(R.reshape(-1, R.shape[-1]).T))


def _chain_operands_t(L, A, R):
    """Operands of the transposed block B01^T (`cy_src/lgmres_cy.pyx:235,241,268`)."""
    Lt = np.transpose(L, (2, 1, 0))
    return (np.ascontiguousarray(Lt.transpose(0, 2, 1).reshape(L.shape[2], -1).T),
            np.ascontiguousarray(np.transpose(A, (0, 2, 1, 3)).reshape(A.shape[0] * A.shape[2], A.shape[1] * A.shape[3]).T),
            np.ascontiguousarray(np.transpose(R, (2, 1, 0)).reshape(-1, R.shape[-1]).T))


def _chain(ops, x2d, r, n, R):
    """The three-dgemm chain `einsum` of `cy_src/lgmres_cy.pyx:126-153`; returns (R*n, r)."""
    Lt, At, Rt = ops
    S = At.shape[0] // n
    s = At.shape[1] // n
    t1 = x2d @ Rt
    t1 = t1.reshape(r, n, R, S).transpose(0, 2, 1, 3).reshape(r * R, n * S)
    t2 = t1 @ At
    t2 = t2.reshape(r, R, s, n).transpose(1, 3, 0, 2).reshape(R * n, r * s)
    return t2 @ Lt


def _unpack(res, r, n, R):
    """`pack_results` (`cy_src/lgmres_cy.pyx:160-174`): (R*n, r) -> flat (r, n, R)."""
    return res.reshape(R, n, r).transpose(2, 1, 0).ravel()


class SchurMatVec:
    """Schur-reduced local KKT operator (`MatVecWrapper.matvec`, `cy_src/lgmres_cy.pyx:291-331`):
    [y; x] -> [B00 y + B01 x ; B21 x - B22 (invI o B01^T y)], evaluated with the same
    dgemm chain and transposes as the reference."""

    keys = ((0, 0), (0, 1), (2, 1), (2, 2))

    def __init__(self, L, A, R, inv_I, shape):
        self.shape = shape
        if T.ALGO is not None:  # one application = the chained local applies
            sh = tuple(shape)
            self.mv_flops = sum(T._path_and_flops(eq, (L[k].shape, A[k].shape, R[k].shape, sh))[1]
                                for eq, k in [("lsr,smnS,LSR,rnR->lmL", k) for k in self.keys]
                                + [("lsr,smnS,LSR,lmL->rnR", (0, 1))])
        self.ops = {k: _chain_operands(L[k], A[k], R[k]) for k in self.keys}
        self.ops_01T = _chain_operands_t(L[0, 1], A[0, 1], R[0, 1])
        r, n, RR = shape
        self.inv_I = np.ascontiguousarray(inv_I.reshape(r * n, RR))

    def _parts(self, v, nb):
        r, n, R = self.shape
        return [np.ascontiguousarray(p) for p in v.reshape(nb, r * n, R)]

    def _schur_x(self, y):
        r, n, R = self.shape
        tmp = _chain(self.ops_01T, y, r, n, R)
        return tmp.reshape(R, n, r).transpose(2, 1, 0).reshape(r * n, R) * self.inv_I

    def _count(self):
        if T.ALGO is not None:
            T.ALGO["flops"] += self.mv_flops
            T.ALGO["calls"] += 1

    def matvec(self, v):
        self._count()
        r, n, R = self.shape
        y, x = self._parts(v, 2)
        res0 = _chain(self.ops[0, 0], y, r, n, R)
        res0 += _chain(self.ops[0, 1], x, r, n, R)
        res1 = _chain(self.ops[2, 1], x, r, n, R)
        res1 -= _chain(self.ops[2, 2], self._schur_x(y), r, n, R)
        return np.concatenate((_unpack(res0, r, n, R), _unpack(res1, r, n, R)))


class IneqSchurMatVec(SchurMatVec):
    """`IneqMatVecWrapper.matvec` (`cy_src/lgmres_cy.pyx:490-510`) on [y; x; t]."""

    keys = ((0, 0), (0, 1), (2, 1), (2, 2), (3, 1), (3, 3))

    def matvec(self, v):
        if INEQ_MATVEC_BUG:
            raise IneqMatvecBug("reference bug: IneqMatVecWrapper.matvec returns a memoryview")
        self._count()
        r, n, R = self.shape
        y, x, t = self._parts(v, 3)
        res0 = _chain(self.ops[0, 0], y, r, n, R)
        res0 += _chain(self.ops[0, 1], x, r, n, R)
        res1 = _chain(self.ops[2, 1], x, r, n, R)
        w = self._schur_x(y)
        w += t
        res1 -= _chain(self.ops[2, 2], w, r, n, R)
        res2 = _chain(self.ops[3, 1], x, r, n, R)
        res2 += _chain(self.ops[3, 3], t, r, n, R)
        return np.concatenate((_unpack(res0, r, n, R), _unpack(res1, r, n, R), _unpack(res2, r, n, R)))


def _fbsub(Lc, b, overwrite_b=False):
    """`forward_backward_sub` (`src/tt_ipm.py:178-181`)."""
    y = sla.solve_triangular(Lc, b, lower=True, check_finite=False, overwrite_b=overwrite_b)
    return sla.solve_triangular(Lc.T, y, lower=False, check_finite=False, overwrite_b=True)


def _report(e):
    tb = traceback.extract_tb(e.__traceback__)
    last = tb[-1] if tb else None
    if last is None:
        print(f"\t⚠️ {type(e).__name__}: {e}")
    else:
        print(f"\t⚠️ {type(e).__name__} in {last.filename},\n\tline {last.lineno}: {last.line.strip()}")


def _local_rhs(Xb_k, b_k, Xb_k1, shape, nb):
    rhs = np.empty(shape)
    for i in range(nb):
        rhs[:, i] = einsum(RHS, Xb_k[i], b_k[i], Xb_k1[i]) if i in b_k else 0
    return rhs


def _run_lgmres(op, rhs_flat, m, rtol):
    restart = min(m, 100)
    aug = max(restart // 10, 3)
    return lgmres(op.matvec, rhs_flat, rtol=rtol, max_it=300, restart=restart, augment=aug)


def local_solver(XAX_k, A_k, XAX_k1, Xb_k, b_k, Xb_k1, prev, size_limit, dense_solve=True, rtol=1e-5):
    """`_ipm_local_solver` (`src/tt_ipm.py:183-282`)."""
    xs = prev.shape
    m = xs[0] * xs[2] * xs[3]
    rhs = _local_rhs(Xb_k, b_k, Xb_k1, xs, 3)
    nrhs = max(np.linalg.norm(rhs), 1e-10)
    inv_I = np.divide(1, einsum(DIAG, XAX_k[1, 2], A_k[1, 2], XAX_k1[1, 2]))
    res_old = np.linalg.norm(A_k.local_product(XAX_k, XAX_k1, prev).__isub__(rhs)) / nrhs
    dense_solve = (np.sqrt(xs[0] * xs[3]) <= size_limit) and dense_solve and (res_old >= rtol)
    failed = not dense_solve
    if dense_solve:
        try:
            rp = rhs[:, 0].reshape(m, 1)
            rd = rhs[:, 1].reshape(m, 1)
            rc = rhs[:, 2].reshape(m, 1)
            LXI = einsum(ASSEMBLE, XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2]).reshape(m, m)
            LXI *= inv_I.reshape(1, -1)
            Leq = einsum(ASSEMBLE, XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1]).reshape(m, m)
            LZ = sla.cholesky(einsum(ASSEMBLE, XAX_k[2, 1], A_k[2, 1], XAX_k1[2, 1]).reshape(m, m),
                              check_finite=False, lower=True, overwrite_a=True)
            b = rp - Leq @ _fbsub(LZ, rc - LXI @ rd, overwrite_b=True)
            Am = _fbsub(LZ, LXI, overwrite_b=True)
            np.matmul(Am, Leq.T, out=Am)  # same BLAS call pattern as the reference (F-ordered out)
            np.matmul(Leq, Am, out=Am)
            Am += einsum(ASSEMBLE, XAX_k[0, 0], A_k[0, 0], XAX_k1[0, 0]).reshape(m, m)
            Am.flat[::Am.shape[1] + 1] += 1e-11
            sol = np.empty(xs)
            sol[:, 0] = sla.solve(Am, b, check_finite=False, overwrite_a=True, overwrite_b=True,
                                  assume_a="gen").reshape(xs[0], xs[2], xs[3])
            sol[:, 2] = ((rd - _apply_t(XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], sol[:, 0]).reshape(-1, 1))
                         * inv_I.reshape(-1, 1)).reshape(xs[0], xs[2], xs[3])
            sol[:, 1] = _fbsub(LZ, rc - _apply(XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], sol[:, 2]).reshape(-1, 1),
                               overwrite_b=True).reshape(xs[0], xs[2], xs[3])
        except Exception as e:
            print(e)
            _report(e)
            failed = True
    if not dense_solve or failed:
        op = SchurMatVec(XAX_k, A_k, XAX_k1, inv_I, (xs[0], xs[2], xs[3]))
        lrhs = np.empty((2, xs[0], xs[2], xs[3]))
        lrhs[0] = rhs[:, 0]
        lrhs[1] = rhs[:, 2]
        lrhs[1] -= _apply(XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], inv_I * rhs[:, 1])
        lnorm = np.linalg.norm(lrhs)
        lvec = op.matvec(np.transpose(prev[:, :2], (1, 0, 2, 3)).flatten()).reshape(2, xs[0], xs[2], xs[3])
        use_prev = np.linalg.norm(lrhs - lvec) < lnorm
        if use_prev:
            lrhs -= lvec
        it_fail = False
        try:
            lsol = _run_lgmres(op, lrhs.flatten(), m, rtol)
        except Exception as e:
            _report(e)
            it_fail = True
            failed = True
            sol = prev
        if not it_fail:
            sol = np.transpose(lsol.reshape(2, xs[0], xs[2], xs[3]), (1, 0, 2, 3))
            if use_prev:
                sol[:, :2] += prev[:, :2]
            z = inv_I * (rhs[:, 1] - _apply_t(XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], sol[:, 0]))
            sol = np.concatenate((sol, z.reshape(xs[0], 1, xs[2], xs[3])), axis=1)
    res_new = np.linalg.norm(A_k.local_product(XAX_k, XAX_k1, sol).__isub__(rhs)) / nrhs
    if res_old < res_new:
        sol = prev
    return sol, res_old, min(res_old, res_new), rhs, nrhs, failed


def local_solver_ineq(XAX_k, A_k, XAX_k1, Xb_k, b_k, Xb_k1, prev, size_limit, dense_solve=True, rtol=1e-5):
    """`_ipm_local_solver_ineq` (`src/tt_ipm.py:284-401`)."""
    xs = prev.shape
    m = xs[0] * xs[2] * xs[3]
    rhs = _local_rhs(Xb_k, b_k, Xb_k1, xs, 4)
    inv_I = np.divide(1, einsum(DIAG, XAX_k[1, 2], A_k[1, 2], XAX_k1[1, 2]))
    nrhs = max(np.linalg.norm(rhs), 1e-10)
    res_old = np.linalg.norm(A_k.local_product(XAX_k, XAX_k1, prev).__isub__(rhs)) / nrhs
    dense_solve = (np.sqrt(xs[0] * xs[3]) <= 0.95 * size_limit) and dense_solve and (res_old >= rtol)
    failed = not dense_solve
    sh3 = (xs[0], xs[2], xs[3])
    if dense_solve:
        try:
            LZ = sla.cholesky(einsum(ASSEMBLE, XAX_k[2, 1], A_k[2, 1], XAX_k1[2, 1]).reshape(m, m),
                              check_finite=False, lower=True, overwrite_a=True)
            rp = rhs[:, 0].reshape(m, 1)
            rd = rhs[:, 1].reshape(m, 1)
            rc = rhs[:, 2].reshape(m, 1)
            rt = rhs[:, 3].reshape(m, 1)
            LZ_rc = _fbsub(LZ, rhs[:, 2].reshape(m, 1))
            LZ_LX = _fbsub(LZ, einsum(ASSEMBLE, XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2]).reshape(m, m), overwrite_b=True)
            Leq = einsum(ASSEMBLE, XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1]).reshape(m, m)
            Top = einsum(ASSEMBLE, XAX_k[3, 1], A_k[3, 1], XAX_k1[3, 1]).reshape(m, m)
            u = rp - Leq @ (LZ_rc - (LZ_LX * inv_I.reshape(1, -1)) @ rd)
            v = rt - Top @ (LZ_rc - (LZ_LX * inv_I.reshape(1, -1)) @ rd)
            Am = einsum(ASSEMBLE, XAX_k[0, 0], A_k[0, 0], XAX_k1[0, 0]).reshape(m, m).__iadd__(
                Leq @ (LZ_LX * inv_I.reshape(1, -1)) @ Leq.T)
            D = einsum(ASSEMBLE, XAX_k[3, 3], A_k[3, 3], XAX_k1[3, 3]).reshape(m, m).__iadd__(Top @ LZ_LX)
            D.flat[::D.shape[1] + 1] += 1e-11
            np.matmul(Top, LZ_LX * inv_I.reshape(1, -1), out=Top)
            np.matmul(Top, Leq.T, out=Top)
            np.matmul(Leq, LZ_LX, out=Leq)
            Dlu, Dpiv = sla.lu_factor(D, check_finite=False, overwrite_a=True)
            rhs_l = u.__isub__(Leq @ sla.lu_solve((Dlu, Dpiv), v, check_finite=False))
            lhs_l = Am.__isub__(Leq.__imatmul__(sla.lu_solve((Dlu, Dpiv), Top, check_finite=False)))
            y = sla.lu_solve(sla.lu_factor(lhs_l, check_finite=False, overwrite_a=True), rhs_l,
                             check_finite=False, overwrite_b=True)
            sol = np.empty(xs)
            sol[:, 0] = y.reshape(sh3)
            sol[:, 3] = sla.lu_solve((Dlu, Dpiv), v.__isub__(Top @ y), check_finite=False, overwrite_b=True).reshape(sh3)
            sol[:, 2] = ((rd - _apply_t(XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], sol[:, 0]).reshape(-1, 1))
                         * inv_I.reshape(-1, 1)).reshape(sh3) - sol[:, 3]
            sol[:, 1] = _fbsub(LZ, rc - _apply(XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], sol[:, 2]).reshape(-1, 1),
                               overwrite_b=True).reshape(sh3)
        except Exception as e:
            _report(e)
            failed = True
    if not dense_solve or failed:
        op = IneqSchurMatVec(XAX_k, A_k, XAX_k1, inv_I, sh3)
        lrhs = np.empty((3,) + sh3)
        lrhs[0] = rhs[:, 0]
        lrhs[1] = rhs[:, 2] - _apply(XAX_k[2, 2], A_k[2, 2], XAX_k1[2, 2], inv_I * rhs[:, 1])
        lrhs[2] = rhs[:, 3]
        lnorm = np.linalg.norm(lrhs)
        lvec = op.matvec(np.transpose(prev[:, [0, 1, 3]], (1, 0, 2, 3)).flatten()).reshape((3,) + sh3)
        use_prev = np.linalg.norm(lrhs - lvec) < lnorm
        if use_prev:
            lrhs -= lvec
        it_fail = False
        try:
            lsol = _run_lgmres(op, lrhs.flatten(), m, rtol)
        except Exception as e:
            _report(e)
            it_fail = True
            failed = True
            sol = prev
        if not it_fail:
            sol = np.transpose(lsol.reshape((3,) + sh3), (1, 0, 2, 3))
            if use_prev:
                sol[:, 0] += prev[:, 0]
                sol[:, 1] += prev[:, 1]
                sol[:, 2] += prev[:, 3]
            z = inv_I * (rhs[:, 1] - _apply_t(XAX_k[0, 1], A_k[0, 1], XAX_k1[0, 1], sol[:, 0])) - sol[:, 2]
            sol = np.concatenate((sol[:, :2], z.reshape(xs[0], 1, xs[2], xs[3]), sol[:, None, 2]), axis=1)
    res_new = np.linalg.norm(A_k.local_product(XAX_k, XAX_k1, sol) - rhs) / nrhs
    if res_old < res_new:
        sol = prev
    return sol, res_old, min(res_old, res_new), rhs, nrhs, failed


# --------------------------------------------------------------------------------------------
# IPM driver (`src/tt_ipm.py:404-1099`)
# --------------------------------------------------------------------------------------------

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


def primal_feasibility(L, b, X, st):
    e = 0.01 * st.eta * st.primal_error_normalisation
    return T.rank_reduce(T.sub(mat_vec_mul(L, T.reshape(X, (4,)), e, st.eps), b), e)


def dual_feasibility(C, Ladj, Z, Y, Tt, st):
    act = st.ineq_status is IneqStatus.ACTIVE
    df = T.rank_reduce(T.sub(T.fast_matrix_vec_mul(Ladj, Y, st.eps),
                             T.rank_reduce(T.add(T.reshape(Z, (4,)), C), st.eps)),
                       st.eps if act else 0.01 * st.eta * st.dual_error_normalisation)
    if act and Tt is not None:
        df = T.rank_reduce(T.sub(df, T.reshape(Tt, (4,))), 0.01 * st.eta * st.dual_error_normalisation)
    return df


def centrality(X, Z, st):
    e = 0.01 * st.eta * st.centrl_error_normalisation
    if st.aho_direction:
        return T.reshape(T.scale(-1, symmetrise(mat_mat_mul(X, Z, e, st.eps), e)), (4,))
    return T.reshape(T.scale(-1, mat_mat_mul(Z, X, e, st.eps)), (4,))


def newton_system(lhs, C, X, Y, Z, Tt, L, Ladj, b, mask, st):
    """`tt_infeasible_newton_system` (`src/tt_ipm.py:429-475`)."""
    rhs = BlockVector()
    pf = primal_feasibility(L, b, X, st)
    st.primal_error = np.divide(T.norm(pf), st.primal_error_normalisation)
    st.is_primal_feasible = np.less(st.primal_error, st.feasibility_tol)
    df = dual_feasibility(C, Ladj, Z, Y, Tt, st)
    st.dual_error = np.divide(T.norm(df), st.dual_error_normalisation)
    st.is_dual_feasible = np.less(st.dual_error, (1 + (st.ineq_status is IneqStatus.ACTIVE)) * st.feasibility_tol)
    st.is_last_iter = st.is_last_iter or (st.is_primal_feasible and st.is_dual_feasible and st.is_central)
    if st.aho_direction:
        lhs[2, 1] = T.psd_rank_reduce(T.scale(0.5, T.add(T.IkronM(Z), T.MkronI(Z))), eps=0.1 * st.eta * st.dual_error_normalisation)
        lhs[2, 2] = T.psd_rank_reduce(T.scale(0.5, T.add(T.MkronI(X), T.IkronM(X))), eps=0.1 * st.eta * st.primal_error_normalisation)
    else:
        lhs[2, 1] = T.psd_rank_reduce(T.MkronI(Z), eps=0.1 * st.eta * st.dual_error_normalisation)
        lhs[2, 2] = T.psd_rank_reduce(T.IkronM(X), eps=0.1 * st.eta * st.primal_error_normalisation)
    if not st.is_primal_feasible or st.is_last_iter:
        rhs[0] = pf
    if not st.is_dual_feasible or st.is_last_iter:
        rhs[1] = df
    if not st.is_central or st.is_last_iter:
        rhs[2] = centrality(X, Z, st)
    if st.ineq_status is IneqStatus.ACTIVE:
        lhs[3, 1] = T.diag_op(Tt, 0.1 * st.eta * st.dual_error_normalisation)
        mX = T.rank_reduce(T.add(T.scale(st.ineq_boundary_val, mask), T.fast_hadamard(mask, X, st.eps)), eps=st.eps)
        lhs[3, 3] = T.rank_reduce(T.add(st.lag_map_t, T.diag_op(mX, st.eps)), eps=0.1 * st.eta * st.dual_error_normalisation)
        if not st.is_central or st.is_last_iter:
            rhs[3] = T.rank_reduce(T.reshape(T.scale(-1, T.fast_hadamard(mX, Tt, st.eps)), (4,)),
                                   eps=0.01 * st.eta * st.centrl_error_normalisation)
    return lhs, rhs, st


def symmetrise(M, e):
    return T.rank_reduce(T.scale(0.5, T.add(M, T.transpose(M))), eps=e)


def psd_symmetrise(M, e):
    return T.psd_rank_reduce(T.scale(0.5, T.add(M, T.transpose(M))), eps=e)


def mask_symmetrise(M, mask, e):
    return T.mask_rank_reduce(T.scale(0.5, T.add(M, T.transpose(M))), mask, eps=e)


def _copy(tt):
    return [np.array(c, copy=True) for c in tt]


def _scale_nd(tt, s):
    if tt is None or np.isclose(s, 1.0):
        return tt
    return T.scale(s, _copy(tt))


def _row_norm(rhs, i):
    row = rhs.get_row(i)
    if row is None:
        return 0.0
    n = T.norm(row)
    return float(n) if np.isfinite(n) else 0.0


def kkt_row_scales(rhs, st):
    """`src/tt_ipm.py:510-528`"""
    eps = max(st.op_tol, 1e-12)
    fn = max(_row_norm(rhs, 0), _row_norm(rhs, 1))
    cn = max(_row_norm(rhs, 2), _row_norm(rhs, 3))
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


def _eff_scale(lhs, key, sc):
    s = sc.get(key[0], 1.0)
    if key in lhs.transposes:
        cr, _ = lhs.transposes[key]
        if cr in sc:
            s = np.sqrt(s * sc[cr])
    if key in lhs.aliases:
        cr, _ = lhs.aliases[key]
        if cr in sc:
            s = np.sqrt(s * sc[cr])
    return float(s)


def row_scaled_kkt(lhs, rhs, st, sc=None):
    """`src/tt_ipm.py:545-568`"""
    if sc is None:
        sc = kkt_row_scales(rhs, st)
    if not sc:
        return lhs, rhs
    L = BlockMatrix()
    L.aliases = dict(lhs.aliases)
    L.transposes = dict(lhs.transposes)
    for key, blk in lhs.data.items():
        L[key] = _scale_nd(blk, _eff_scale(lhs, key, sc))
    R = BlockVector()
    for i in rhs.keys():
        R[i] = _scale_nd(rhs.get_row(i), sc.get(i, 1.0))
    if st.verbose:
        print(f"KKT row scaling: feas={sc.get(0, sc.get(1, 1.0)):.2e}, cent={sc.get(2, sc.get(3, 1.0)):.2e}", flush=True)
    return L, R


def _ineq_step(Att, Dtt, e_tt, st):
    """`src/tt_ipm.py:730-747`"""
    s = T.add(Att, Dtt)
    if st.compl_ineq_mask:
        s = T.add(s, st.compl_ineq_mask)
    s = T.rank_reduce(s, st.eps)
    e_tt, _ = min_eig(T.diag_op(s, st.eps), x0=e_tt, tol=1e-8, verbose=st.verbose)
    esq = T.reshape(e_tt, (2, 2))
    if np.abs(T.inner(s, esq)) > st.eps:
        esq = T.normalise(T.fast_hadamard(esq, esq, st.eps))
        mA = np.abs(T.inner(Att, esq))
        mD = T.inner(Dtt, esq)
        step = 1 if mD >= -st.eps else np.clip(-mA / mD, a_min=0, a_max=1)
    else:
        step = 1
    return step, e_tt


def _ineq_step_sizes(xs, zs, X, Tt, DX, DT, mask, st):
    """`src/tt_ipm.py:750-779`"""
    if xs > 0:
        mX = T.fast_hadamard(mask, X, st.eps)
        mDX = T.fast_hadamard(mask, DX, st.eps)
        xis, st.eigen_xt0 = _ineq_step(T.add(mX, T.scale(st.ineq_boundary_val, mask)), T.scale(xs, mDX), st.eigen_xt0, st)
        if not st.is_last_iter:
            if 1 - xis < st.op_tol and T.norm(Tt) < st.op_tol:
                if st.ineq_status is IneqStatus.ACTIVE:
                    st.ineq_status = IneqStatus.SETTING_INACTIVE
            else:
                if st.ineq_status is IneqStatus.INACTIVE:
                    st.ineq_status = IneqStatus.SETTING_ACTIVE
        xs *= xis
    if zs > 0 and st.ineq_status is IneqStatus.ACTIVE:
        ts, st.eigen_zt0 = _ineq_step(Tt, T.scale(zs, DT), st.eigen_zt0, st)
        zs *= ts
    return xs, zs


def step_sizes(X, Z, Tt, DX, DZ, DT, mask, st):
    """`src/tt_ipm.py:700-727`"""
    if st.is_last_iter:
        X = T.add(X, T.scale(st.boundary_val, T.identity(len(X))))
        Z = T.add(Z, T.scale(st.boundary_val, T.identity(len(Z))))
    xs, st.eigen_x0 = max_generalised_eigen(X, DX, x0=st.eigen_x0, tol=1e-8, verbose=st.verbose)
    zs, st.eigen_z0 = max_generalised_eigen(Z, DZ, x0=st.eigen_z0, tol=1e-8, verbose=st.verbose)
    if st.ineq_status is not IneqStatus.NOT_IN_USE:
        if st.is_last_iter:
            X = T.add(X, T.scale(st.ineq_boundary_val + st.boundary_val, mask))
            Tt = T.add(Tt, T.scale(st.ineq_boundary_val + st.boundary_val, mask))
        xs, zs = _ineq_step_sizes(xs, zs, X, Tt, DX, DT, mask, st)
    tau = 0.9 + 0.05 * min(xs, zs)
    if st.verbose:
        print("Step search concluded.")
        print(f"Step sizes: a_p:{xs:.2e}, a_d:{zs:.2e}", flush=True)
    return tau * xs, tau * zs


def newton_step(lhs, rhs, mask, X, Z, Tt, ZX, TX, st, solver):
    """`_tt_ipm_newton_step` (`src/tt_ipm.py:571-697`)."""
    try:
        sc = kkt_row_scales(rhs, st)
        Lp, Rp = row_scaled_kkt(lhs, rhs, st, sc)
        Dl, _ = solver(Lp, Rp, st.mals_delta0, st.kkt_iterations + st.is_last_iter, st.mals_rank_restriction, st.eta)
        st.mals_delta0 = Dl
        DX = symmetrise(T.reshape(get_block(1, Dl), (2, 2)), st.eps)
        DZ = symmetrise(T.reshape(get_block(2, Dl), (2, 2)), st.eps)
        DY = T.rank_reduce(get_block(0, Dl), eps=st.eps)
        DT = None
        if st.ineq_status is IneqStatus.ACTIVE:
            DT = T.rank_reduce(get_block(3, Dl), eps=st.eps)
            DT = T.fast_hadamard(mask, T.reshape(DT, (2, 2)), st.eps)
        xs, zs = step_sizes(X, Z, Tt, DX, DZ, DT, mask, st)
        if not st.is_central and not st.is_last_iter:
            DXZ = T.inner(DX, DZ)
            if st.ineq_status is IneqStatus.ACTIVE:
                mu_aff = (ZX + xs * zs * DXZ + zs * T.inner(X, DZ) + xs * T.inner(DX, Z)
                          + TX + xs * zs * T.inner(DT, DX)
                          + zs * (T.inner(X, DT) + st.ineq_boundary_val * T.entrywise_sum(DT))
                          + xs * T.inner(DX, Tt))
                e = max(1, 3 * min(xs, zs) ** 2)
                st.sigma = min(0.99, max(mu_aff / (ZX + TX), 0) ** e)
                if st.sigma > 1e-4:
                    rhs[3] = T.rank_reduce(T.add(T.scale(st.sigma * st.mu, T.reshape(mask, (4,))), rhs.get_row(3)),
                                           0.1 * st.eta * st.centrl_error_normalisation)
            else:
                mu_aff = ZX + xs * zs * DXZ + zs * T.inner(X, DZ) + xs * T.inner(DX, Z)
                e = max(1, 3 * min(xs, zs) ** 2)
                st.sigma = min(0.99, max(mu_aff / ZX, 0) ** e)
            ce = 0.1 * st.eta * st.centrl_error_normalisation
            if DXZ > 0.1 * st.centrality_tol:
                term = centrality(DX, DZ, st)
                if st.sigma > 1e-4:
                    rhs[2] = T.rank_reduce(T.add(T.scale(st.sigma * st.mu, T.reshape(T.identity(len(X)), (4,))),
                                                 T.add(rhs.get_row(2), term)), ce)
                else:
                    rhs[2] = T.rank_reduce(T.add(rhs.get_row(2), term), ce)
            else:
                if st.sigma > 1e-4:
                    rhs[2] = T.rank_reduce(T.add(T.scale(st.sigma * st.mu, T.reshape(T.identity(len(X)), (4,))),
                                                 rhs.get_row(2)), ce)
                else:
                    rhs[2] = rhs.get_row(2)
            Lc, Rc = row_scaled_kkt(lhs, rhs, st, sc)
            Dc, _ = solver(Lc, Rc, st.mals_delta0, st.kkt_iterations + st.is_last_iter, st.mals_rank_restriction, st.eta)
            st.mals_delta0 = Dc
            DXc = symmetrise(T.reshape(get_block(1, Dc), (2, 2)), st.eps)
            DZc = symmetrise(T.reshape(get_block(2, Dc), (2, 2)), st.eps)
            DYc = T.rank_reduce(get_block(0, Dc), eps=st.eps)
            DX = T.rank_reduce(T.add(DXc, DX), eps=st.eps)
            DY = T.rank_reduce(T.add(DYc, DY), eps=st.eps)
            DZ = T.rank_reduce(T.add(DZc, DZ), eps=st.eps)
            if st.ineq_status is IneqStatus.ACTIVE:
                DTc = T.rank_reduce(get_block(3, Dc), eps=st.eps)
                DTc = T.fast_hadamard(mask, T.reshape(DTc, (2, 2)), st.eps)
                DT = T.rank_reduce(T.add(DTc, DT), eps=st.eps)
            xs, zs = step_sizes(X, Z, Tt, DX, DZ, DT, mask, st)
        else:
            st.sigma = 0
    except Exception as e:
        print(f"\n\t⚠️ Attention: {e}")
        print("\n\t==> Full traceback (most recent call last):")
        traceback.print_exc(file=sys.stdout)
        return 0, 0, None, None, None, None, st
    return xs, zs, DX, DY, DZ, DT, st


def _initialise(mask, st, dim, lam, lam_ineq):
    X = T.scale(lam, T.identity(dim))
    Z = T.scale(lam, T.identity(dim))
    Y = T.reshape(T.zero_matrix(dim), (4,))
    Tt = None
    if st.ineq_status is IneqStatus.ACTIVE:
        Tt = T.scale(lam_ineq, mask)
        xs, _ = max_generalised_eigen(X, mask, tol=1e-7, verbose=st.verbose)
        X = T.rank_reduce(T.add(X, T.scale(0.1 * xs, mask)), 0.1 * st.eta * st.primal_error_normalisation)
    return X, Y, Z, Tt


def _stalled(prev, st, gap_tol):
    if st.is_last_iter:
        return False
    return (abs(prev['primal'] - st.primal_error) < 0.04 * gap_tol
            and abs(prev['dual'] - st.dual_error) < 0.04 * gap_tol
            and abs(prev['centrality'] - st.centrality_error) < 0.02 * gap_tol)


def _check_convergence(st, fin, ZX, TX, abs_tol, max_ref):
    if not st.is_last_iter:
        return st, fin
    if abs(ZX) + abs(TX) < abs_tol and st.primal_error < abs_tol and st.dual_error < abs_tol:
        fin = 0
    else:
        fin -= 1
        st.boundary_val = 0.001 * (1 - (fin / max_ref))
        if fin == 1:
            st.kkt_iterations += 1
    return st, fin


def tt_ipm(lag_maps, obj_tt, lin_op_tt, bias_tt, ineq_mask=None, max_iter=100, max_refinement=5,
           warm_up=3, gap_tol=1e-4, aho_direction=True, op_tol=1e-5, abs_tol=8e-4, eps=1e-12,
           mals_restarts=3, r_max=1000, lambdaStar=1, lambdaStarIneq=1, epsilonDash=None,
           epsilonDashineq=None, verbose=False, trace=None):
    """`tt_ipm` (`src/tt_ipm.py:901-1099`).  `trace` (list) collects one record per Newton
    system assembly: mu, errors, sigma, ranks (SURVEY.md §8(c) golden-trace schema)."""
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        return _tt_ipm(lag_maps, obj_tt, lin_op_tt, bias_tt, ineq_mask, max_iter, max_refinement, warm_up,
                       gap_tol, aho_direction, op_tol, abs_tol, eps, mals_restarts, r_max, lambdaStar,
                       lambdaStarIneq, verbose, trace)


def _tt_ipm(lag_maps, C, L, b, mask, max_iter, max_ref, warm_up, gap_tol, aho, op_tol, abs_tol, eps,
            restarts, r_max, lam, lam_ineq, verbose, trace):
    dim = len(C)
    st = IPMStatus(len(C), 2 * gap_tol, gap_tol / np.sqrt(dim), op_tol, eps, aho, False, np.inf, False,
                   np.inf, False, np.inf, np.inf, False,
                   IneqStatus.NOT_IN_USE if mask is None else IneqStatus.ACTIVE, verbose, 1, 1, r_max)
    lag_maps = {k: T.rank_reduce(v, eps=eps) for k, v in lag_maps.items()}
    C = T.rank_reduce(C, eps=eps)
    L = T.rank_reduce(L, eps=eps)
    b = T.rank_reduce(b, eps=eps)
    st.primal_error_normalisation = 1 + T.norm(b)
    st.dual_error_normalisation = 1 + T.norm(C)
    skel = BlockMatrix()
    skel[1, 2] = T.reshape(T.identity(2 * dim), (4, 4))

    def make_solver(ls):
        return lambda lhs, rhs, x0, nswp, restr, tol: restarted_block_amen(
            lhs, rhs, rank_restriction=restr, x0=x0, local_solver=ls, op_tol=op_tol, termination_tol=tol,
            num_restarts=restarts, inner_m=nswp, verbose=verbose)

    solver_ineq = make_solver(local_solver_ineq)
    solver_eq = make_solver(local_solver)
    if st.ineq_status is IneqStatus.ACTIVE:
        solver = solver_ineq
        st.num_ineq_constraints = T.inner(mask, mask)
        st.compl_ineq_mask = T.rank_reduce(T.sub(T.one_matrix(dim), mask), eps=eps)
        st.lag_map_t = lag_maps["t"]
        skel.add_alias((1, 2), (1, 3))
    else:
        solver = solver_eq
        st.num_ineq_constraints = 0
    Ladj = T.transpose(L)
    skel[0, 1] = T.scale(-1, L)
    skel.add_alias((0, 1), (1, 0), is_transpose=True)
    skel[0, 0] = lag_maps["y"]
    st.lag_map_y = lag_maps["y"]
    X, Y, Z, Tt = _initialise(mask, st, dim, lam, lam_ineq)
    it = 0
    fin = max_ref
    prev = {'primal': np.inf, 'dual': np.inf, 'centrality': np.inf}
    lhs = skel
    while fin > 0:
        it += 1
        st.aho_direction = (it > warm_up)
        if max_iter - max_ref == it - 1 and not st.is_last_iter:
            print("============================================\n Maximum #iterations reached!\n"
                  "============================================")
            st.is_last_iter = True
        ZX = T.inner(Z, X)
        TX = (T.inner(X, Tt) + st.ineq_boundary_val * T.entrywise_sum(Tt)) if st.ineq_status is IneqStatus.ACTIVE else 0
        st.mu = np.divide(abs(ZX) + abs(TX), (2 ** dim + (st.ineq_status is IneqStatus.ACTIVE) * st.num_ineq_constraints))
        st.centrl_error_normalisation = 1 + abs(T.inner(C, T.reshape(X, (4,))))
        st.centrality_error = st.mu / st.centrl_error_normalisation
        st.is_central = np.less(st.centrality_error, st.centrality_tol)
        st.eta = max(min(st.eta, 2 * st.mu), st.op_tol)
        lhs_m, rhs_v, st = newton_system(lhs, C, X, Y, Z, Tt, L, Ladj, b, mask, st)
        if trace is not None:
            trace.append({"iter": it, "mu": float(st.mu), "primal_error": float(st.primal_error),
                          "dual_error": float(st.dual_error), "centrality_error": float(st.centrality_error),
                          "sigma": float(st.sigma), "ranksX": T.ranks(X), "ranksZ": T.ranks(Z),
                          "ranksY": T.ranks(Y), "is_last_iter": bool(st.is_last_iter)})
        if verbose:
            print(f"\n--- Iteration {it - 1} ---")
            print(f"Errors: Centrality={st.centrality_error:.4e}, Primal={st.primal_error:.4e}, Dual={st.dual_error:.4e}")
            print(f"Ranks: X={T.ranks(X)}, Z={T.ranks(Z)}, Y={T.ranks(Y)}", flush=True)
        st, fin = _check_convergence(st, fin, ZX, TX, abs_tol, max_ref)
        if fin == 0:
            it -= 1
            break
        xs, zs, DX, DY, DZ, DT, st = newton_step(lhs_m, rhs_v, mask, X, Z, Tt, ZX, TX, st, solver)
        if (DX is None and DZ is None) or (xs < 1e-5 and zs < 1e-5):
            if st.is_last_iter:
                break
            print("============================================\n Hit PSD boundary! Entering finishing phase.\n"
                  "============================================")
            st.is_last_iter = True
        else:
            e_p = 0.1 * st.eta * st.primal_error_normalisation
            e_d = 0.1 * st.eta * st.dual_error_normalisation
            X = symmetrise(T.add(X, T.scale(xs, DX)), e_p) if fin <= 1 else psd_symmetrise(T.add(X, T.scale(xs, DX)), e_p)
            Z = symmetrise(T.add(Z, T.scale(zs, DZ)), e_d) if fin <= 1 else psd_symmetrise(T.add(Z, T.scale(zs, DZ)), e_d)
            Y = T.rank_reduce(T.add(Y, T.scale(zs, DY)), st.eps)
            Y = T.reshape(symmetrise(T.reshape(T.sub(Y, T.fast_matrix_vec_mul(st.lag_map_y, Y, st.eps)), (2, 2)), e_d), (4,))
            if st.ineq_status is IneqStatus.ACTIVE:
                if fin <= 1:
                    Tt = symmetrise(T.add(Tt, T.scale(zs, DT)), e_d)
                else:
                    Tt = mask_symmetrise(T.add(Tt, T.scale(zs, DT)), mask, e_d)
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
        if _stalled(prev, st, gap_tol):
            st.is_last_iter = True
        prev['primal'] = st.primal_error
        prev['dual'] = st.dual_error
        prev['centrality'] = st.centrality_error
    info = {"num_iters": it, "ranksX": T.ranks(X), "ranksY": T.ranks(Y), "ranksZ": T.ranks(Z),
            "ranksT": T.ranks(Tt) if Tt else [0] * (st.dim - 1), "status": st}
    return X, Y, Tt, Z, info
