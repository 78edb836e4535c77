"""Pin the CPU oracle (`oracle/`) against golden vectors produced by the reference itself
(`tests/golden/make_golden.py`).  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import tt as T
from oracle import als as A
from oracle import ipm as I

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "prims.npz"))


def _tt(key):
    return [G[f"{key}/{i}"].copy() for i in range(int(G[key + "/n"]))]


def _dense(tt):
    t = tt[0]
    for c in tt[1:]:
        t = np.tensordot(t, c, axes=(-1, 0))
    return np.sum(t, axis=(0, -1))


def _close(a, b, rtol=1e-12):
    scale = max(np.max(np.abs(b)), 1e-300)
    assert np.max(np.abs(a - b)) <= rtol * scale, np.max(np.abs(a - b)) / scale


@pytest.mark.parametrize("ci", range(5))
def test_rank_reduce(ci):
    tt = _tt(f"round{ci}/in")
    eps = float(G[f"round{ci}/eps"])
    res = T.rank_reduce([c.copy() for c in tt], eps)
    assert T.ranks(res) == list(G[f"round{ci}/ranks"])
    _close(_dense(res), G[f"round{ci}/dense"])
    if f"round{ci}/psd_dense" in G:
        res = T.psd_rank_reduce([c.copy() for c in tt], eps)
        assert T.ranks(res) == list(G[f"round{ci}/psd_ranks"])
        _close(_dense(res), G[f"round{ci}/psd_dense"])


@pytest.mark.parametrize("ci", range(3))
def test_zipup_products(ci):
    Am, x, M1, M2 = (_tt(f"zip{ci}/{k}") for k in ("A", "x", "M1", "M2"))
    eps = float(G[f"zip{ci}/eps"])
    mv = T.fast_matrix_vec_mul(Am, x, eps)
    assert T.ranks(mv) == list(G[f"zip{ci}/mv_ranks"])
    _close(_dense(mv), G[f"zip{ci}/mv_dense"])
    mm = T.fast_mat_mat_mul(M1, M2, eps)
    assert T.ranks(mm) == list(G[f"zip{ci}/mm_ranks"])
    _close(_dense(mm), G[f"zip{ci}/mm_dense"])
    _close(_dense(T.fast_hadamard(M1, M2, eps)), G[f"zip{ci}/had_dense"])
    _close(np.array(T.inner(M1, M2)), G[f"zip{ci}/ip"])


@pytest.mark.parametrize("ci", range(3))
def test_environment_and_apply(ci):
    g = {k: G[f"env{ci}/{k}"] for k in ("P", "xl", "A", "Q", "v", "b", "Pb", "Qb")}
    _close(A.phi_fwd_A(g["P"], g["xl"], g["A"], g["xl"]), G[f"env{ci}/fwd"])
    _close(A.phi_bck_A(g["Q"], g["xl"], g["A"], g["xl"]), G[f"env{ci}/bck"])
    _close(A.phi_fwd_rhs(g["Pb"], g["b"], g["xl"]), G[f"env{ci}/fwd_rhs"])
    _close(A.phi_bck_rhs(g["Qb"], g["b"], g["xl"]), G[f"env{ci}/bck_rhs"])
    _close(I._apply(g["P"], g["A"], g["Q"], g["v"]), G[f"env{ci}/apply"])
    _close(I._apply_t(g["P"], g["A"], g["Q"], g["v"]), G[f"env{ci}/apply_t"])
    _close(T.einsum(I.RHS, g["Pb"], g["b"], g["Qb"]), G[f"env{ci}/local_rhs"])


@pytest.mark.parametrize("ci", range(3))
def test_schur_matvec(ci):
    keys = [(0, 0), (0, 1), (2, 1), (2, 2)]
    L = {k: G[f"mv{ci}/L{k[0]}{k[1]}"] for k in keys}
    Am = {k: G[f"mv{ci}/A{k[0]}{k[1]}"] for k in keys}
    R = {k: G[f"mv{ci}/R{k[0]}{k[1]}"] for k in keys}
    invI = G[f"mv{ci}/invI"]
    r, n, RR = invI.shape
    op = I.SchurMatVec(L, Am, R, invI, (r, n, RR))
    y = op.matvec(G[f"mv{ci}/x"])
    _close(y, G[f"mv{ci}/y"], 1e-13)


@pytest.mark.parametrize("ci", range(3))
def test_mask_rank_reduce(ci):
    res = T.mask_rank_reduce(_tt(f"mask{ci}/in"), _tt(f"mask{ci}/mask"), float(G[f"mask{ci}/eps"]))
    assert T.ranks(res) == list(G[f"mask{ci}/ranks"])
    _close(_dense(res), G[f"mask{ci}/dense"])


@pytest.mark.parametrize("ci", range(3))
def test_rank_retraction(ci):
    res = T.rank_retraction(_tt(f"retract{ci}/in"), [int(u) for u in G[f"retract{ci}/upper"]])
    assert T.ranks(res) == list(G[f"retract{ci}/ranks"])
    _close(_dense(res), G[f"retract{ci}/dense"])


@pytest.mark.parametrize("ci", range(3))
def test_ineq_schur_matvec(ci):
    """3-block operator (`cy_src/lgmres_cy.pyx:490-510`, fixed mode) against the reference's output"""
    keys = [(0, 0), (0, 1), (2, 1), (2, 2), (3, 1), (3, 3)]
    L = {k: G[f"imv{ci}/L{k[0]}{k[1]}"] for k in keys}
    Am = {k: G[f"imv{ci}/A{k[0]}{k[1]}"] for k in keys}
    R = {k: G[f"imv{ci}/R{k[0]}{k[1]}"] for k in keys}
    invI = G[f"imv{ci}/invI"]
    op = I.IneqSchurMatVec(L, Am, R, invI, invI.shape)
    _close(op.matvec(G[f"imv{ci}/x"]), G[f"imv{ci}/y"], 1e-13)


def test_normalise_rng_coupling():
    np.random.seed(7)
    res = T.normalise(_tt("norm/in"), radius=np.sqrt(10))
    _close(_dense(res), G["norm/dense"])
    assert np.random.randint(0, 1 << 30) == int(G["norm/next_randint"])


def test_prune_singular_vals_rule():
    s = np.array([3.0, 1.0, 1e-3, 1e-7])
    assert T.prune_singular_vals(s, 1e-2) == 2
    assert T.prune_singular_vals(s, 1e-9) == 4
    assert T.prune_singular_vals(np.zeros(3), 1.0) == 1
    assert T.prune_singular_vals(s, 100.0) == 1


RUNS = json.load(open(os.path.join(HERE, "golden", "runs.json")))


_ORACLE_RUN = """
import json, sys
import numpy as np
import yaml
sys.path.insert(0, sys.argv[1])
from oracle.problems import run_and_record
cfg = yaml.safe_load(open(sys.argv[2]))
trace = []
r = run_and_record("maxcut", cfg, int(sys.argv[3]), int(sys.argv[4]), trace=trace)
conv = lambda o: o.item() if isinstance(o, np.generic) else (o.tolist() if isinstance(o, np.ndarray) else str(o))
print(json.dumps({"trace": trace, "r": r}, default=conv))
"""


@pytest.mark.parametrize("key", ["maxcut_5_r1_s0", "maxcut_5_r1_s319"])
def test_oracle_full_run_maxcut5(key):
    """Whole TT-IPM on maxcut_5 (configs[0]): the oracle must follow one of the reference's own runs
    (golden or twins) within 50x the reference's rounding noise -- the same policy the device's
    whole-solve parity tests apply (tests/parity_policy.py).  The oracle's path, like the reference's
    (hence its PYTHONHASHSEED twins), depends on the interpreter's string-hash seed through set /
    dict iteration order, so it runs in a child process under PYTHONHASHSEED=0: with a random seed
    the test was flaky -- hash seeds 0-30 on s319: 28 follow the golden or one of its three committed
    twins, 3 take a branch no committed reference run takes."""
    import subprocess
    import sys

    from tests.parity_policy import check_against_reference_runs
    g = RUNS[key]
    root = os.path.join(HERE, "..")
    env = dict(os.environ, PYTHONHASHSEED="0", OPENBLAS_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-c", _ORACLE_RUN, root, os.path.join(root, "configs", g["config"] + ".yaml"),
                          str(g["seed"]), str(g["rank"])], env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    name, per, cum = check_against_reference_runs(key, res["trace"], res["r"])
    print(key, "follows", name, ["%.0e" % v for v in per])


@pytest.mark.parametrize("hash_seed", [16, 24, 29])
def test_oracle_maxcut5_hash_seed_departures(hash_seed):
    """The hash seeds test_oracle_full_run_maxcut5 does not run (the pinned seed must not
    hide them).  Over PYTHONHASHSEED 0..30 the oracle's maxcut_5 s319 run follows one of the committed
    unmodified reference runs (golden, _h2, _h3) on 28 seeds; on these three it takes a contraction
    order no committed reference run took and leaves them by more than 50x their noise
    (profiles/r06_oracle_hash_scan_s319.txt) -- at the end-point level only: same iteration count, gap within 3e-5
    relative of the golden's.  Asserted as such, so a change that makes them depart further fails."""
    import subprocess
    import sys

    from tests.parity_policy import check_against_reference_runs
    key = "maxcut_5_r1_s319"
    g = RUNS[key]
    root = os.path.join(HERE, "..")
    env = dict(os.environ, PYTHONHASHSEED=str(hash_seed), OPENBLAS_NUM_THREADS="1")
    out = subprocess.run([sys.executable, "-c", _ORACLE_RUN, root, os.path.join(root, "configs", g["config"] + ".yaml"),
                          str(g["seed"]), str(g["rank"])], env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    with pytest.raises(AssertionError):
        check_against_reference_runs(key, res["trace"], res["r"])
    assert res["r"]["num_iters"] == g["num_iters"]
    assert abs(res["r"]["gap"] - g["gap"]) <= 3e-5 * g["gap"], (res["r"]["gap"], g["gap"])


class _Bounded(Exception):
    pass


@pytest.mark.parametrize("key", sorted(k for k in RUNS if RUNS[k].get("bounded")))
def test_oracle_bounded_trace(key):
    """Bounded reference traces (fixed-mode inequality configs): the oracle's first Newton-system
    assemblies, AMEn solution ranks and step sizes against the reference's."""
    import yaml
    from oracle.problems import run_and_record
    g = RUNS[key]
    n = int(g["bounded"])
    amen, steps = [], []

    class Trace(list):
        def append(self, item):
            super().append(item)
            if len(self) >= n:
                raise _Bounded

    o_amen, o_steps = I.restarted_block_amen, I.step_sizes

    def h_amen(*a, **k):
        sol, res = o_amen(*a, **k)
        amen.append([int(c.shape[-1]) for c in sol[:-1]])
        return sol, res

    def h_steps(*a, **k):
        xs, zs = o_steps(*a, **k)
        steps.append([float(xs), float(zs)])
        return xs, zs

    cfg = yaml.safe_load(open(os.path.join(HERE, "..", "configs", g["config"] + ".yaml")))
    trace = Trace()
    I.restarted_block_amen, I.step_sizes = h_amen, h_steps
    try:
        with pytest.raises(_Bounded):
            run_and_record(g["problem"], cfg, g["seed"], g["rank"], trace=trace)
    finally:
        I.restarted_block_amen, I.step_sizes = o_amen, o_steps
    for i, (a, b) in enumerate(zip(trace, g["trace"])):
        assert a["ranksX"] == b["ranksX"], (i, a["ranksX"], b["ranksX"])
        for k in ("mu", "primal_error", "dual_error", "centrality_error"):
            assert abs(a[k] - b[k]) <= 1e-6 * abs(b[k]) + 1e-14, (i, k, a[k], b[k])
    # the AMEn solutions' TT ranks may differ by directions carrying rounding-level energy (measured:
    # solve 7 keeps [1,2,..,3] where the reference keeps [1,3,..,3]) without moving the iterates
    assert len(amen) == len(g["amen"])
    assert np.allclose(steps, g["steps"], rtol=1e-6, atol=1e-12)


AP = np.load(os.path.join(HERE, "golden", "approx.npz"))


@pytest.mark.parametrize("name", ["mm0", "mv0", "mm1"])
def test_approx_products(name):
    """oracle ALS approximate products vs the reference's (same seed): ranks, draws, tensor."""
    a = [AP[f"{name}/a/{i}"].copy() for i in range(int(AP[f"{name}/a/n"]))]
    b = [AP[f"{name}/b/{i}"].copy() for i in range(int(AP[f"{name}/b/n"]))]
    np.random.seed(int(AP[f"{name}/seed"]))
    fn = A.approx_mat_mat_mul if b[0].ndim == 4 else A.approx_mat_vec_mul
    res = fn(a, b, tol=float(AP[f"{name}/tol"]))
    assert np.random.randint(0, 1 << 30) == int(AP[f"{name}/next_randint"])
    assert T.ranks(res) == list(AP[f"{name}/ranks"])
    t = res[0]
    for c in res[1:]:
        t = np.tensordot(t, c, axes=(-1, 0))
    _close(t, AP[f"{name}/dense"], 1e-10)


# ---- dense local KKT solves (src/tt_ipm.py:183-401; fixtures: tests/golden/make_local.py)
from tests import local_cases as LC  # noqa: E402


def _oracle_case(name):
    def setb(bm, k, a):
        bm[k] = [a]
    return LC.load(name, lambda a: np.array(a, copy=True), A.BlockMatrix, lambda bm: A.CoreView(bm, 0), setb,
                   lambda bm, k1, k2, t: bm.add_alias(k1, k2, t))


@pytest.mark.parametrize("name", LC.CASES)
def test_local_solver_matches_reference(name, capsys):
    """the oracle's `_ipm_local_solver(_ineq)` against the reference's own recorded calls: right-hand
    side, norms and old residual to 1e-12; the dense solutions to 1e-10; the failure flag and the
    exception class the reference printed; LGMRES fallbacks (PETSc restatement on both sides) to 1e-8."""
    args, ex = _oracle_case(name)
    import warnings
    f = I.local_solver_ineq if LC.is_ineq(name) else I.local_solver
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # as in the reference's IPM (src/tt_ipm.py:16)
        sol, res_old, res_min, rhs, nrhs, failed = f(*args)
    out = capsys.readouterr().out
    assert failed == ex["failed"]
    if ex["exc"]:
        assert f"⚠️ {ex['exc']} in" in out, out
    assert LC.rel(rhs, ex["rhs"]) <= 1e-12
    assert abs(nrhs - ex["nrhs"]) <= 1e-12 * ex["nrhs"]
    assert abs(res_old - ex["res_old"]) <= 1e-10 * ex["res_old"]
    if name.endswith("_ill"):
        # the LGMRES fallback on the ill-conditioned operator stalls (res_min ~0.8) and its iterate
        # is rounding-chaotic: only the keep-prev rule is checked
        assert res_min <= res_old
        return
    tol = 1e-10 if not ex["failed"] else 1e-8
    assert LC.rel(sol, ex["sol"]) <= tol, LC.rel(sol, ex["sol"])
    # the new residual of a dense solve sits at rounding level (||A x - rhs|| / ||rhs|| ~ 1e-10, set
    # by summation order): compared in absolute terms there
    assert abs(res_min - ex["res_min"]) <= max(1e-6 * ex["res_min"], 1e-9)


def test_extra_departure_floor_rule():
    """The floor under a KNOWN_EXTRA_DEPARTURES xfail: following the named bounded
    twin of the reference passes, a trace that leaves it (or a non-finite end point) fails."""
    import copy

    from tests.parity_policy import (BOUNDED_TWINS, EXTRA_DEPARTURE_FOLLOWS, KNOWN_EXTRA_DEPARTURES, RUNS,
                                     check_extra_departure_floor)
    # every KNOWN_EXTRA_DEPARTURES key has a floor: a named bounded twin (EXTRA_DEPARTURE_FOLLOWS) or
    # full unmodified twins for check_extra_follow_floor (tests/test_parity_policy.py)
    full = {k for k in KNOWN_EXTRA_DEPARTURES if any(k + x in RUNS for x in ("_t8", "_h1", "_h2", "_h3"))}
    assert set(EXTRA_DEPARTURE_FOLLOWS) <= set(KNOWN_EXTRA_DEPARTURES)
    assert set(EXTRA_DEPARTURE_FOLLOWS) | full == set(KNOWN_EXTRA_DEPARTURES)
    end = {"gap": 2.0, "feas": 1e-3}
    for key, (twin, n, tol) in EXTRA_DEPARTURE_FOLLOWS.items():
        t = BOUNDED_TWINS[f"{key}_{twin}"]["trace"]
        check_extra_departure_floor(key, copy.deepcopy(t), end)
        off = copy.deepcopy(t)
        k0 = next(iter(off[n - 1]))
        off[n - 1][k0] = off[n - 1][k0] * (1 + 100 * tol) + 100 * tol
        with pytest.raises(AssertionError):
            check_extra_departure_floor(key, off, end)
        with pytest.raises(AssertionError):
            check_extra_departure_floor(key, copy.deepcopy(t), {"gap": float("nan"), "feas": 1e-3})
        with pytest.raises(AssertionError):
            check_extra_departure_floor(key, copy.deepcopy(t)[:n - 1], end)
