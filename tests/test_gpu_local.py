"""Rows a6 / a7 against the reference's own output: the device `_ipm_local_solver(_ineq)` -- whose
dense branch is ONE `ttk_dense_schur_solve(_ineq)` call -- on local KKT solves recorded from the
reference (`tests/golden/local.npz`, `tests/golden/make_local.py`: maxcut_10 s41 and corr_clust_9
s764 fixed, plus the reference's Cholesky-failure and ill-conditioned cases built from them).

Tolerances: right-hand side 1e-12, ||rhs|| and the old residual 1e-10 (device reduction order),
dense solutions 1e-10 relative to the largest entry (fp64 LU / Cholesky of m <= 288 systems in
another summation order), the failure flag and the exception class exactly."""
import numpy as np
import pytest

from tests import local_cases as LC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ttipm_amd import dev as D
    from ttipm_amd import _lib
    assert _lib.lib is not None
    return D


def _device_case(D, name):
    from ttipm_amd import tt_als as TA

    def setb(bm, k, a):
        bm[k] = [a]
    return LC.load(name, D.from_numpy, TA.TTBlockMatrix, lambda bm: bm[0], setb,
                   lambda bm, k1, k2, t: bm.add_alias(k1, k2, t))


@pytest.mark.parametrize("name", LC.CASES)
def test_local_solver_matches_reference(dev, name, capsys):
    import warnings
    from ttipm_amd import tt_ipm
    D = dev
    args, ex = _device_case(D, name)
    f = tt_ipm._ipm_local_solver_ineq if LC.is_ineq(name) else tt_ipm._ipm_local_solver
    l0 = D.lib.ttk_launch_count()
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        sol, res_old, res_min, rhs, nrhs, failed = f(*args)
    assert D.lib.ttk_launch_count() > l0
    out = capsys.readouterr().out
    assert failed == ex["failed"], (failed, ex["failed"], out)
    if ex["exc"]:
        assert f"⚠️ {ex['exc']} in" in out, out
    assert LC.rel(D.read(rhs), ex["rhs"]) <= 1e-12
    assert abs(nrhs - ex["nrhs"]) <= 1e-10 * ex["nrhs"]
    assert abs(res_old - ex["res_old"]) <= 1e-10 * ex["res_old"]
    if name.endswith("_ill"):  # LGMRES stalls on the ill-conditioned operator: keep-prev rule only
        assert res_min <= res_old
        return
    tol = 1e-10 if not ex["failed"] else 1e-7  # LGMRES fallbacks: device vs restated PETSc reductions
    assert LC.rel(D.read(sol), ex["sol"]) <= tol, LC.rel(D.read(sol), ex["sol"])
    # a direct solve's new residual is at the rounding floor (~1e-10 of ||rhs||, set by summation
    # order): absolute there
    assert abs(res_min - ex["res_min"]) <= max(1e-6 * ex["res_min"], 1e-9)


@pytest.mark.parametrize("name", [c for c in LC.CASES if "_dense" in c or c.endswith(("_chol", "_ill"))])
def test_native_dense_status_matches_reference(dev, name):
    """`ttk_dense_schur_solve(_ineq)` called directly: the solution on the reference's dense
    successes, the reference's exception class (LinAlgError for a failed Cholesky, LinAlgWarning for
    dgecon's rcond < eps) on its failures."""
    from ttipm_amd import tt_ipm
    D = dev
    args, ex = _device_case(D, name)
    XAX_k, A_k, XAX_k1, Xb_k, b_k, Xb_k1, prev = args[:7]
    xs = tuple(prev.shape)
    rhs = D.from_numpy(ex["rhs"])
    inv_I = D.recip(tt_ipm.einsum(tt_ipm.DIAG, XAX_k[1, 2], A_k[1, 2], XAX_k1[1, 2]))
    f = tt_ipm._dense_native_ineq if LC.is_ineq(name) else tt_ipm._dense_native
    if ex["exc"]:
        with pytest.raises(Exception) as ei:
            f(XAX_k, A_k, XAX_k1, rhs, inv_I, xs)
        assert type(ei.value).__name__ == ex["exc"]
    else:
        got = D.read(f(XAX_k, A_k, XAX_k1, rhs, inv_I, xs))
        assert LC.rel(got, ex["sol"]) <= 1e-10
