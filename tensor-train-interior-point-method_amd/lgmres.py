"""Device LGMRES with PETSc KSPLGMRES semantics (drop-in for `LGMRESSolver`,
`src/tt_ipm.py:101-162`).

The Krylov basis, Hessenberg matrices and Givens rotations live on the device
(`ttk_lgmres_*` kernels); the host runs PETSc's integer bookkeeping (restart cycles,
augmentation order) and reads one residual estimate per Arnoldi step for the convergence test
(KSPConvergedDefault).  The algorithm is restated in `oracle/petsc_lgmres.py`."""
import ctypes

import numpy as np

from . import dev as D
from ._lib import lib

CONVERGED_RTOL, CONVERGED_ATOL = 2, 3
DIVERGED_NULL, DIVERGED_ITS, DIVERGED_DTOL, DIVERGED_BREAKDOWN, DIVERGED_NANORINF = -2, -3, -4, -5, -9


class PetscConvFailed(RuntimeError):
    """KSPLGMRESBuildSoln: HH(it,it) is identically zero (PETSC_ERR_CONV_FAILED)."""


def _hh_size(max_k):
    ld = max_k + 1
    return 2 * (max_k + 2) * ld + (max_k + 2) + 2 * ld + 8


def _grs_offset(max_k):
    ld = max_k + 1
    return 2 * (max_k + 2) * ld


def lgmres(matvec_into, b, rtol=1e-8, max_it=300, restart=30, augment=2, abstol=1e-50, dtol=1e5,
           haptol=1e-30, info=None):
    """Solve A x = b from x0 = 0.  `matvec_into(v, out)` writes A v into `out` (device, 1-D)."""
    n = b.numel()
    max_k = int(restart)
    aug_dim = int(augment)
    x = D.zeros(n)
    V = D.empty(max_k + 1, n)
    hh = D.zeros(_hh_size(max_k))
    grs0 = hh[_grs_offset(max_k):_grs_offset(max_k) + 1]
    nd = max(aug_dim, 1)
    augvecs = D.empty(nd, n)
    a_augvecs = D.empty(nd, n)
    aug_temp = D.empty(n)
    aug_order = np.zeros(nd, dtype=np.int64)
    aug_ct = 0
    its = 0
    itcount = 0
    reason = 0
    state = {}
    guess_zero = True
    res = 0.0
    s = D._stream()
    resbuf = (ctypes.c_double * 2)()
    flags = (ctypes.c_int * 2)()

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
            D.copy_(V[0], b)
        else:
            matvec_into(x, V[0])
            D.copy_(V[0], b, 1.0, -1.0)  # r = b - A x
        it_arnoldi = max_k - aug_dim
        it_total = it_arnoldi + aug_ct
        res = D.norm(V[0])
        D.fill_(grs0, res)
        if res == 0.0:
            reason = CONVERGED_ATOL
            break
        D.copy_(V[0], V[0], 1.0 / res)
        reason = converged(its, res)
        loc_it = 0
        hapend = False
        last_diag = 1.0
        while (not reason) and loc_it < it_total and its < max_it:
            if loc_it < it_arnoldi:
                matvec_into(V[loc_it], V[loc_it + 1])
            else:
                order = loc_it - it_arnoldi + 1
                spot = 0
                for ii in range(aug_dim):
                    if aug_order[ii] == order:
                        spot = ii
                        break
                D.copy_(V[loc_it + 1], a_augvecs[spot])
            D.check(lib.ttk_lgmres_arnoldi_sync(s, V.data_ptr(), n, loc_it, hh.data_ptr(), max_k, haptol,
                                                resbuf, flags), "lgmres_arnoldi")
            hapend = bool(flags[0])
            if flags[1]:
                reason = DIVERGED_NULL
                break
            res = resbuf[0]
            last_diag = resbuf[1]
            loc_it += 1
            its += 1
            reason = converged(its, res)
            if hapend and not reason:
                reason = DIVERGED_BREAKDOWN
                break
        cycle_its = loc_it
        it = loc_it - 1
        built = False
        if it >= 0:
            ita = max_k - aug_dim
            if ita >= it + 1:
                it_aug = 0
                ita = it + 1
            else:
                it_aug = (it + 1) - ita
            if last_diag == 0.0:
                raise PetscConvFailed("HH(it,it) is identically zero; it = %d" % it)
            ptrs = [V[j].data_ptr() for j in range(ita)]
            for ii in range(it_aug):
                spot = 0
                for jj in range(aug_dim):
                    if aug_order[jj] == ii + 1:
                        spot = jj
                        break
                ptrs.append(augvecs[spot].data_ptr())
            arr = (ctypes.c_void_p * len(ptrs))(*ptrs)
            D.check(lib.ttk_lgmres_build(s, hh.data_ptr(), max_k, it, arr, len(ptrs), n, x.data_ptr(),
                                         aug_temp.data_ptr()), "lgmres_build")
            built = True
        if (not reason) and its < max_it and aug_dim > 0 and built:
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
            aug_order[:aug_dim] += 1
            aug_order[spot] = 1
            D.check(lib.ttk_lgmres_aug(s, hh.data_ptr(), max_k, it_total, V.data_ptr(), n, 0.0,
                                       aug_temp.data_ptr(), augvecs[spot].data_ptr(), a_augvecs[spot].data_ptr()),
                    "lgmres_aug")
        itcount += cycle_its
        if itcount >= max_it:
            if not reason:
                reason = DIVERGED_ITS
            break
        guess_zero = False
    if info is not None:
        info.update(reason=reason, its=its, res=res)
    return x
