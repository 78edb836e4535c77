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


def test_oracle_full_run_maxcut5():
    """Whole TT-IPM on maxcut_5 seed 0: oracle vs the reference's own run (same LGMRES restatement)."""
    import yaml
    from oracle.problems import run_and_record
    g = RUNS["maxcut_5_r1_s0"]
    cfg = yaml.safe_load(open(os.path.join(HERE, "..", "configs", g["config"] + ".yaml")))
    trace = []
    r = run_and_record("maxcut", cfg, g["seed"], g["rank"], trace=trace)
    assert r["num_iters"] == g["num_iters"]
    assert r["ranksX"] == g["ranksX"] and r["ranksZ"] == g["ranksZ"]
    for k in ("gap", "feas", "dual_feas"):
        assert abs(r[k] - g[k]) <= 1e-4 * abs(g[k]), (k, r[k], g[k])
    for a, b in zip(trace, g["trace"]):
        assert a["ranksX"] == b["ranksX"]
        assert abs(a["mu"] - b["mu"]) <= 1e-5 * abs(b["mu"])


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
