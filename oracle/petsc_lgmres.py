"""CPU restatement of PETSc's KSPLGMRES (TEST INFRASTRUCTURE -- checker only, never shipped).

The reference solves its iterative local KKT systems with petsc4py
(`src/tt_ipm.py:101-154`): `KSP.setType('lgmres')`, options `-ksp_gmres_restart`,
`-ksp_lgmres_augment`, `-ksp_rtol`, `-ksp_max_it`, shell (MATPYTHON) operator, zero initial
guess, no preconditioner (PETSc's default PC for a shell matrix with no factorisation or
diagonal-block support is PCNONE).  PETSc 3.25.1 / petsc4py 3.25.1 (`env.yaml:13-14`) is not in
this image, so its published algorithm is restated here:

* `KSPSolve_LGMRES`   (src/ksp/ksp/impls/gmres/lgmres/lgmres.c): restart loop, zero guess on
  the first cycle (no matvec), true residual `b - A x` on later cycles.
* `KSPLGMRESCycle`: `it_arnoldi = max_k - aug_dim` (approx_constant off),
  `it_total = it_arnoldi + aug_ct`; Arnoldi steps then augmentation steps that re-use the
  stored `A*augvec`; classical Gram-Schmidt without refinement
  (`KSPGMRESClassicalGramSchmidtOrthogonalization`, cgstype REFINE_NEVER); happy-breakdown
  tolerance `haptol = 1e-30`.
* `KSPLGMRESUpdateHessenberg`: Givens rotations applied to HH, GRS.
* `KSPLGMRESBuildSoln`: back substitution on HH, solution from Krylov + augmentation vectors,
  AUG_TEMP kept for the next augmentation vector; `A*augvec = V (HES y)`.
* `KSPConvergedDefault`: `ttol = max(rtol*||r0||, abstol)`, divergence at `dtol*||r0||`.

Parity of this restatement against real PETSc is UNPINNED (no reference fixture pins PETSc;
the stale `tests/test_tt_preprocessing.py:25-36` only solves a 2x2 system to 1e-10).  The GPU
LGMRES in the product follows the same algorithm and is pinned against this restatement.
"""
import os

import numpy as np

# Reduction kernels.  The default restatement uses NumPy/BLAS reductions (np.dot, gemv).  Real
# PETSc's rounding differs from both the restatement and the device at that level: VecNorm_Seq is
# BLAS dnrm2 (scaled sum of squares), VecMDot_Seq sums x[i]*y[i] in index order per vector, and
# VecMAXPY_Seq adds the vectors in groups of 4 (the nv % 4 remainder first).  GOLDEN_PETSC_KERNELS=1
# (tests/golden/make_golden.py's `_p<H>` twins) restates those kernels, so the reference can be re-run
# under PETSc-like reduction orders: the spread of those twins is reference rounding noise that the
# restatement alone cannot show.  Test infrastructure only.
PETSC_KERNELS = os.environ.get("GOLDEN_PETSC_KERNELS") == "1"


def _norm(v):
    if PETSC_KERNELS:
        from scipy.linalg import blas
        return float(blas.dnrm2(v))
    return float(np.sqrt(np.dot(v, v)))


def _mdot(V, w):
    """h_j = <V_j, w>"""
    if PETSC_KERNELS:
        return np.array([np.cumsum(vj * w)[-1] for vj in V]) if len(V) else np.zeros(0)
    return V @ w


def _maxpy_into(x, coef, V):
    """x += sum_j coef_j V_j in VecMAXPY_Seq's order (the nv % 4 remainder group, then groups of 4,
    each group's terms summed before it is added to x)"""
    nv = len(coef)
    r = nv & 3
    if r:
        acc = coef[0] * V[0]
        for j in range(1, r):
            acc = acc + coef[j] * V[j]
        x += acc
    for j in range(r, nv, 4):
        x += coef[j] * V[j] + coef[j + 1] * V[j + 1] + coef[j + 2] * V[j + 2] + coef[j + 3] * V[j + 3]
    return x


def _maxpy_sum(coef, V):
    """sum_j coef_j V_j (VecSet(0) + VecMAXPY when PETSC_KERNELS)"""
    if not PETSC_KERNELS:
        return coef @ V
    return _maxpy_into(np.zeros(V.shape[1]), coef, V)


CONVERGED_RTOL = 2
CONVERGED_ATOL = 3
DIVERGED_NULL = -2
DIVERGED_ITS = -3
DIVERGED_DTOL = -4
DIVERGED_BREAKDOWN = -5
DIVERGED_NANORINF = -9


class PetscConvFailed(RuntimeError):
    """Mirrors PETSc's PETSC_ERR_CONV_FAILED raised by KSPLGMRESBuildSoln (HH(it,it)==0)."""


def lgmres(matvec, b, rtol=1e-8, max_it=300, restart=30, augment=2,
           abstol=1e-50, dtol=1e5, haptol=1e-30, info=None):
    """Solve A x = b with x0 = 0, PETSc LGMRES semantics.  Returns x (new array)."""
    b = np.asarray(b, dtype=np.float64).ravel()
    n = b.size
    max_k = int(restart)
    aug_dim = int(augment)
    x = np.zeros(n)
    its = 0
    itcount = 0
    reason = 0
    aug_ct = 0
    aug_order = np.zeros(max(aug_dim, 1), dtype=np.int64)
    augvecs = np.zeros((max(aug_dim, 1), n))
    a_augvecs = np.zeros((max(aug_dim, 1), n))
    # Hessenberg storage, zero-initialised once per solve (PetscCalloc in KSPSetUp_LGMRES)
    HH = np.zeros((max_k + 2, max_k + 1))
    HES = np.zeros((max_k + 2, max_k + 1))
    GRS = np.zeros(max_k + 2)
    CC = np.zeros(max_k + 1)
    SS = np.zeros(max_k + 1)
    state = {"rnorm0": None, "ttol": None}
    guess_zero = True
    nmatvec = 0

    def converged(k, rnorm):
        if k == 0:
            state["rnorm0"] = rnorm
            state["ttol"] = max(rtol * rnorm, abstol)
        if rnorm != rnorm or np.isinf(rnorm):
            return DIVERGED_NANORINF
        if rnorm <= state["ttol"]:
            return CONVERGED_ATOL if rnorm < abstol else CONVERGED_RTOL
        if rnorm >= dtol * state["rnorm0"]:
            return DIVERGED_DTOL
        return 0

    while not reason:
        if guess_zero:
            r = b.copy()
        else:
            r = b - matvec(x)
            nmatvec += 1
        # ---------------- KSPLGMRESCycle ----------------
        it_arnoldi = max_k - aug_dim
        it_total = it_arnoldi + aug_ct
        V = np.zeros((it_total + 1, n))
        V[0] = r
        res = _norm(r)
        GRS[0] = res
        if res == 0.0:
            reason = CONVERGED_ATOL
            cycle_its = 0
            break
        V[0] *= 1.0 / res
        reason = converged(its, res)
        loc_it = 0
        hapend = False
        while (not reason) and loc_it < it_total and its < max_it:
            if loc_it < it_arnoldi:
                V[loc_it + 1] = matvec(V[loc_it])
                nmatvec += 1
            else:
                order = loc_it - it_arnoldi + 1
                spot = 0
                for ii in range(aug_dim):
                    if aug_order[ii] == order:
                        spot = ii
                        break
                V[loc_it + 1] = a_augvecs[spot]
            # classical Gram-Schmidt, no refinement
            h = _mdot(V[:loc_it + 1], V[loc_it + 1])
            if PETSC_KERNELS:  # VecMAXPY(w, it+1, -h, V)
                _maxpy_into(V[loc_it + 1], -h, V[:loc_it + 1])
            else:
                V[loc_it + 1] -= h @ V[:loc_it + 1]
            HH[:loc_it + 1, loc_it] = h
            HES[:loc_it + 1, loc_it] = h
            tt = _norm(V[loc_it + 1])
            HH[loc_it + 1, loc_it] = tt
            HES[loc_it + 1, loc_it] = tt
            hapbnd = abs(tt / GRS[loc_it])
            if hapbnd > haptol:
                hapbnd = haptol
            if tt > hapbnd:
                V[loc_it + 1] *= 1.0 / tt
            else:
                hapend = True
            # KSPLGMRESUpdateHessenberg
            for j in range(1, loc_it + 1):
                t0 = HH[j - 1, loc_it]
                HH[j - 1, loc_it] = CC[j - 1] * t0 + SS[j - 1] * HH[j, loc_it]
                HH[j, loc_it] = CC[j - 1] * HH[j, loc_it] - SS[j - 1] * t0
            if not hapend:
                hv = HH[loc_it, loc_it]
                hv1 = HH[loc_it + 1, loc_it]
                tr = np.sqrt(hv * hv + hv1 * hv1)
                if tr == 0.0:
                    reason = DIVERGED_NULL
                    break
                CC[loc_it] = hv / tr
                SS[loc_it] = hv1 / tr
                GRS[loc_it + 1] = -(SS[loc_it] * GRS[loc_it])
                GRS[loc_it] = CC[loc_it] * GRS[loc_it]
                HH[loc_it, loc_it] = CC[loc_it] * hv + SS[loc_it] * hv1
                res = abs(GRS[loc_it + 1])
            else:
                res = 0.0
            loc_it += 1
            its += 1
            reason = converged(its, res)
            if hapend and not reason:
                reason = DIVERGED_BREAKDOWN
                break
        cycle_its = loc_it
        # ---------------- KSPLGMRESBuildSoln(GRS, x, x, it = loc_it-1) ----------------
        it = loc_it - 1
        aug_temp = None
        if it >= 0:
            ita = max_k - aug_dim
            if ita >= it + 1:
                it_aug = 0
                ita = it + 1
            else:
                it_aug = (it + 1) - ita
            if HH[it, it] == 0.0:
                raise PetscConvFailed("HH(it,it) is identically zero; it = %d" % it)
            GRS[it] = GRS[it] / HH[it, it]
            for k in range(it - 1, -1, -1):
                t0 = GRS[k]
                for j in range(k + 1, it + 1):
                    t0 = t0 - HH[k, j] * GRS[j]
                GRS[k] = t0 / HH[k, k]
            temp = _maxpy_sum(GRS[:ita], V[:ita])
            for ii in range(it_aug):
                spot = 0
                for jj in range(aug_dim):
                    if aug_order[jj] == ii + 1:
                        spot = jj
                        break
                temp = temp + GRS[ita + ii] * augvecs[spot]
            aug_temp = temp
            x = x + temp
        # ---------------- augmentation vector bookkeeping ----------------
        if (not reason) and its < max_it and aug_dim > 0 and aug_temp is not None:
            if aug_ct == 0:
                spot = 0
                aug_ct += 1
            elif aug_ct < aug_dim:
                spot = aug_ct
                aug_ct += 1
            else:
                spot = 0
                for ii in range(aug_dim):
                    if aug_order[ii] == aug_dim:
                        spot = ii
            nrm = _norm(aug_temp)
            inv = 1.0 / nrm
            augvecs[spot] = aug_temp * inv
            aug_order[:aug_dim] += 1
            aug_order[spot] = 1
            avec = np.zeros(it_total + 1)
            for ii in range(it_total + 1):
                for jj in range(0, min(ii + 2, it_total + 1)):
                    avec[jj] += HES[jj, ii] * GRS[ii]
            a_augvecs[spot] = _maxpy_sum(avec, V[:it_total + 1]) * inv
        itcount += cycle_its
        if itcount >= max_it:
            if not reason:
                reason = DIVERGED_ITS
            break
        guess_zero = False
    if info is not None:
        info["reason"] = reason
        info["its"] = its
        info["matvecs"] = nmatvec
        info["res"] = res
    return x
