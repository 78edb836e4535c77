"""Device LGMRES with PETSc KSPLGMRES semantics (drop-in for `LGMRESSolver`,
`src/tt_ipm.py:101-162`).

The Krylov basis, Hessenberg matrices and Givens rotations live on the device
(`ttk_lgmres_*` kernels); the host runs PETSc's integer bookkeeping (restart cycles,
augmentation order) and reads one residual estimate per Arnoldi step for the convergence test
(KSPConvergedDefault).  The algorithm is restated in `oracle/petsc_lgmres.py`.

Host syncs: Arnoldi steps are enqueued in speculative chunks of up to CHUNK steps
(`ttk_lgmres_arnoldi_async`); the device stops modifying the Krylov state at the first step that
meets a stop condition, and the host replays the per-step test on the chunk's records after ONE
read, so decisions, iteration counts and iterates are those of the step-by-step loop."""
import ctypes
import os

import numpy as np

from . import dev as D
from ._lib import lib

CONVERGED_RTOL, CONVERGED_ATOL = 2, 3
DIVERGED_NULL, DIVERGED_ITS, DIVERGED_DTOL, DIVERGED_BREAKDOWN, DIVERGED_NANORINF = -2, -3, -4, -5, -9


CHUNK = int(os.environ.get("TTIPM_LGMRES_CHUNK", "8"))


class PetscConvFailed(RuntimeError):
    """KSPLGMRESBuildSoln: HH(it,it) is identically zero (PETSC_ERR_CONV_FAILED)."""


# with a native Schur operator the whole solve is one library call (ttk_lgmres: the same kernel
# sequence as the loop below, host bookkeeping in C++)
NATIVE_SOLVE = os.environ.get("TTIPM_LGMRES_NATIVE", "1") == "1"


class _Info(ctypes.Structure):
    _fields_ = [("reason", ctypes.c_int), ("its", ctypes.c_int), ("res", ctypes.c_double), ("matvecs", ctypes.c_int)]


def _lgmres_native(handle, b, rtol, max_it, max_k, aug_dim, info):
    from ._lib import TTK_ERR_NOT_CONVERGED
    b = D.contig(b)
    n = b.numel()
    x = D.empty(n)
    st = _Info()
    s = D._stream()
    rc = lib.ttk_lgmres(D.ctx(), int(handle), b.data_ptr(), x.data_ptr(), n, max_k, aug_dim,
                        float(rtol), int(max_it), CHUNK, ctypes.byref(st))
    if rc == TTK_ERR_NOT_CONVERGED:
        raise PetscConvFailed(lib.ttk_last_error().decode())
    D.check(rc, "lgmres")
    del s
    if info is not None:
        info.update(reason=st.reason, its=st.its, res=st.res, matvecs=st.matvecs, native_matvecs=st.matvecs)
    return x


def _hh_size(max_k):
    ld = max_k + 1
    return 2 * (max_k + 2) * ld + (max_k + 2) + 2 * ld + 8


def _grs_offset(max_k):
    ld = max_k + 1
    return 2 * (max_k + 2) * ld


def lgmres(matvec_into, b, rtol=1e-8, max_it=300, restart=30, augment=2, abstol=1e-50, dtol=1e5,
           haptol=1e-30, info=None, native=0):
    """Solve A x = b from x0 = 0.  `matvec_into(v, out)` writes A v into `out` (device, 1-D);
    `native`: a ttk_schur_build handle of the same operator, so whole Arnoldi chunks run in one
    native call (`ttk_lgmres_chunk`) instead of a Python loop per step."""
    n = b.numel()
    max_k = int(restart)
    aug_dim = int(augment)
    if native and NATIVE_SOLVE and abstol == 1e-50 and dtol == 1e5 and haptol == 1e-30:
        return _lgmres_native(native, b, rtol, max_it, max_k, aug_dim, info)
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
    nmv_native = 0
    nmv = 0  # operator applications the algorithm consumed (speculative chunk steps past a stop excluded)
    s = D._stream()
    resbuf = (ctypes.c_double * 2)()
    flags = (ctypes.c_int * 2)()
    ctl = D.zeros(1 + 5 * max(CHUNK, 1))

    def _matvec_or_aug(li):
        if li < it_arnoldi:
            matvec_into(V[li], V[li + 1])
        else:
            order = li - it_arnoldi + 1
            spot = 0
            for ii in range(aug_dim):
                if aug_order[ii] == order:
                    spot = ii
                    break
            D.copy_(V[li + 1], a_augvecs[spot])

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
            nmv += 1
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
            kmax = min(CHUNK, it_total - loc_it, max_it - its)
            in_native = False
            if kmax <= 1:
                _matvec_or_aug(loc_it)
                D.check(lib.ttk_lgmres_arnoldi_sync(s, V.data_ptr(), n, loc_it, hh.data_ptr(), max_k, haptol,
                                                    resbuf, flags), "lgmres_arnoldi")
                recs = [(float(its + 1), resbuf[0], float(flags[0]), float(flags[1]), resbuf[1])]
            else:
                ttol, divtol = state["ttol"], dtol * state["rnorm0"]
                in_native = bool(native and loc_it + kmax <= it_arnoldi)
                if in_native:  # whole chunk in one native call
                    D.check(lib.ttk_lgmres_chunk(s, native, V.data_ptr(), n, loc_it, kmax, hh.data_ptr(), max_k,
                                                 haptol, ttol, divtol, ctl.data_ptr(), float(its + 1)),
                            "lgmres_chunk")
                else:
                    for q in range(kmax):
                        _matvec_or_aug(loc_it + q)
                        D.check(lib.ttk_lgmres_arnoldi_async(s, V.data_ptr(), n, loc_it + q, hh.data_ptr(), max_k,
                                                             haptol, ttol, divtol, ctl.data_ptr(), q,
                                                             float(its + q + 1)), "lgmres_arnoldi")
                h = D.read(ctl[:1 + 5 * kmax])
                recs = [tuple(h[1 + 5 * q:6 + 5 * q]) for q in range(kmax)]
            for q, (marker, r_, hap_, null_, diag_) in enumerate(recs):
                if marker != its + 1:
                    raise RuntimeError(f"lgmres: device stopped the Arnoldi chunk at step {its} without a "
                                       "host-side stop reason")
                hapend = bool(hap_)
                if null_:
                    reason = DIVERGED_NULL
                    break
                res = r_
                last_diag = diag_
                nmv += loc_it < it_arnoldi
                nmv_native += kmax > 1 and in_native
                loc_it += 1
                its += 1
                reason = converged(its, res)
                if hapend and not reason:
                    reason = DIVERGED_BREAKDOWN
                    break
                if reason:
                    break
            if reason == DIVERGED_NULL or reason == DIVERGED_BREAKDOWN:
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
        info.update(reason=reason, its=its, res=res, matvecs=nmv, native_matvecs=nmv_native)
    return x
