"""Loader for tests/golden/step.npz (tests/golden/make_step.py): the reference's own step-size
eigen-ALS calls (`tt_max_generalised_eigen`, src/tt_als.py:1132-1283) and every two-site local solve
inside them (`_step_size_local_solve`, :931-1038), recorded on maxcut_10 seeds 14 and 41.

TEST INFRASTRUCTURE (shared by the oracle's CPU test and the device's GPU test)."""
import os

import numpy as np

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "step.npz")
F = np.load(PATH)
CASES = [str(c) for c in F["cases"]]
LOCAL_ARGS = ("p1", "p2", "XAX_k", "A_k", "A_kp1", "XAX_k2", "XDX_k", "D_k", "D_kp1", "XDX_k2", "step",
              "size_limit", "trunc_tol", "eps", "max_rank", "bwd")

# Local solves whose output ranks the device does not share with the reference on the reference's
# own inputs (r06_step_fixture.log).  Every step size agrees (<= 4e-14); these local eigenproblems
# have degenerate smallest eigenvalues (clusters of 6 .. 168 equal eigenvalues, `tools/step_clusters.py`),
# where the reference's ARPACK returns the Krylov vector grown from v0 = the previous solution and the
# device its exact dense eigenvector: both are eigenvectors of the same eigenvalue, whose unfoldings
# truncate to different ranks at trunc_tol = 1e-8 / sqrt(d).
DEVICE_RANK_DEPARTURES = {"s14_c17": {5, 12, 13, 14}, "s14_c19": {4}}


def tt(name):
    if name + "/n" not in F:
        return None
    return [F[f"{name}/{i}"].copy() for i in range(int(F[name + "/n"]))]


def rng_state(prefix):
    return ("MT19937", F[prefix + "/key"], int(F[prefix + "/pos"]), int(F[prefix + "/g"]), float(F[prefix + "/c"]))


def call(c):
    """(A, Delta, x0, rng_state, reference step, reference solution TT)"""
    return tt(c + "/A"), tt(c + "/Delta"), tt(c + "/x0"), rng_state(c + "/rng"), float(F[c + "/step"]), tt(c + "/x")


def nlocal(c):
    return int(F[c + "/nlocal"])


def local(c, j):
    """(args tuple of `_step_size_local_solve` without bwd, bwd, rng_state, expected dict)"""
    p = f"{c}/l{j}"
    a = [F[f"{p}/{k}"] for k in LOCAL_ARGS]
    args = [np.array(v) for v in a[:10]] + [float(a[10]), int(a[11]), float(a[12]), float(a[13]), int(a[14])]
    exp = {"s1": F[p + "/s1"], "s2": F[p + "/s2"], "step": float(F[p + "/step_out"]), "res": float(F[p + "/res"])}
    return args, bool(a[15]), rng_state(p + "/rng"), exp


def product(s1, s2):
    return np.einsum("rny,ytR->rntR", s1, s2)
