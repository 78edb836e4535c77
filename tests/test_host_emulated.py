"""Product HOST logic (einsum planner, TT algebra, AMEn sweeps, LGMRES bookkeeping, IPM control
flow) on CPU, with the libttk C ABI replaced by the NumPy emulator in tests/emu_ttk.py.  The GPU
run of the same path is tests/test_gpu_parity.py; this file checks the host side alone against
the reference golden runs."""
import json
import os

import pytest
import yaml

from tests.emu_ttk import emulated_ttipm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = json.load(open(os.path.join(ROOT, "tests", "golden", "runs.json")))


@pytest.fixture(scope="module")
def pkg():
    return emulated_ttipm()


def test_maxcut_5_seed0_matches_reference(pkg):
    from ttipm_amd.utils import run_and_record
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "maxcut_5.yaml")))
    trace = []
    r = run_and_record("maxcut", cfg, 0, 1, trace=trace, verbose=False)
    g = GOLD["maxcut_5_r1_s0"]
    assert r["num_iters"] == g["num_iters"]
    assert r["ranksX"] == g["ranksX"] and r["ranksZ"] == g["ranksZ"]
    assert r["gap"] == pytest.approx(g["gap"], rel=1e-4)
    assert r["feas"] == pytest.approx(g["feas"], rel=1e-3)
    for a, b in zip(trace, g["trace"]):
        assert a["ranksX"] == b["ranksX"]
        assert a["mu"] == pytest.approx(b["mu"], rel=1e-4)


def test_shard_pack_roundtrip(pkg):
    import numpy as np
    from ttipm_amd import shard
    from ttipm_amd.utils import create
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "maxcut_5.yaml")))
    prep = create("maxcut", cfg, 319, 1, verbose=False)
    meta, flat = shard.pack(prep)
    back = shard.unpack(meta, flat)
    for k in ("C", "L", "b"):
        assert len(back[k]) == len(prep[k])
        for a, b in zip(back[k], prep[k]):
            assert tuple(a.shape) == tuple(b.shape) and bool((a == b).all())
    for k in prep["lag"]:
        for a, b in zip(back["lag"][k], prep["lag"][k]):
            assert bool((a == b).all())
    s0, s1 = prep["rng_state"], back["rng_state"]
    assert s0[0] == s1[0] and np.array_equal(s0[1], s1[1]) and s0[2:] == s1[2:]


APPROX = os.path.join(ROOT, "tests", "golden", "approx.npz")


def _approx_case(name):
    import numpy as np
    f = np.load(APPROX)
    tt = lambda k: [f[f"{name}/{k}/{i}"].copy() for i in range(int(f[f"{name}/{k}/n"]))]  # noqa: E731
    return f, tt("a"), tt("b")


def _dense(tt):
    import numpy as np
    t = tt[0]
    for c in tt[1:]:
        t = np.tensordot(t, c, axes=(-1, 0))
    return t


@pytest.mark.parametrize("name", ["mm0", "mv0", "mm1"])
def test_approx_products_match_reference(pkg, name):
    """ALS approximate products (`src/tt_als.py:1502-1762`, taken when a rank product exceeds the
    exact limits 40/80): device host logic vs the reference's outputs (tests/golden/approx.npz),
    same MT19937 stream (ranks, draw count and the represented tensor)."""
    import numpy as np
    from ttipm_amd import dev as D
    from ttipm_amd import tt_als as A
    f, a, b = _approx_case(name)
    np.random.seed(int(f[f"{name}/seed"]))
    fn = A.tt_approx_mat_mat_mul if b[0].ndim == 4 else A.tt_approx_mat_vec_mul
    got = fn([D.from_numpy(c) for c in a], [D.from_numpy(c) for c in b], tol=float(f[f"{name}/tol"]))
    assert np.random.randint(0, 1 << 30) == int(f[f"{name}/next_randint"])
    got = [D.read(c) for c in got]
    assert [c.shape[-1] for c in got[:-1]] == list(f[f"{name}/ranks"])
    want = f[f"{name}/dense"]
    assert np.max(np.abs(_dense(got) - want)) <= 1e-9 * np.max(np.abs(want))


@pytest.mark.parametrize("gen,largest,n,maxiter", [(False, False, 60, 100), (True, True, 60, 100),
                                                   (False, False, 400, 20), (True, True, 400, 20)])
def test_lobpcg_matches_scipy(pkg, gen, largest, n, maxiter):
    """device single-vector LOBPCG (tt_eig.lobpcg) vs scipy.sparse.linalg.lobpcg with warnings as
    errors (the reference's setting): same outcome (converged / raises), same eigenvalue."""
    import warnings
    import numpy as np
    import scipy.sparse.linalg as spla
    from ttipm_amd import dev as D
    from ttipm_amd import tt_eig as E
    rng = np.random.RandomState(n + 7 * gen)
    Q, _ = np.linalg.qr(rng.randn(n, n))
    A = (Q * np.linspace(1.0, 40.0, n)) @ Q.T
    Bm = None
    if gen:
        Bq, _ = np.linalg.qr(rng.randn(n, n))
        Bm = (Bq * np.linspace(1.0, 3.0, n)) @ Bq.T
    x0 = rng.randn(n, 1)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        try:
            lam_ref, v_ref = spla.lobpcg(A, x0.copy(), B=Bm, tol=1e-8, largest=largest, maxiter=maxiter)
            ref_ok = True
        except UserWarning:
            ref_ok = False
    Ad = D.from_numpy(A)
    Bd = D.from_numpy(Bm) if gen else None
    opA = lambda v: D.matmul(Ad, v.view(-1, 1)).view(-1)  # noqa: E731
    opB = (lambda v: D.matmul(Bd, v.view(-1, 1)).view(-1)) if gen else None  # noqa: E731
    try:
        lam, v = E.lobpcg(opA, D.from_numpy(x0.reshape(-1)), B=opB, tol=1e-8, largest=largest, maxiter=maxiter)
        ok = True
    except E.LobpcgFailure:
        ok = False
    assert ok == ref_ok
    if ok:
        assert abs(lam - float(lam_ref[0])) <= 1e-10 * abs(float(lam_ref[0]))


def test_concurrent_solves_in_threads_match_one_at_a_time(pkg):
    """bench.py's solves in flight within one process: slot threads, each with a private NumPy
    random stream (`ttipm_amd.rng`) and its own per-thread device state (`dev._TL`, the eigen
    sweep's deferred residuals, the constant cores), give every seed exactly its one-at-a-time
    result."""
    import threading

    from ttipm_amd import rng
    from ttipm_amd.utils import create, solve
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", "maxcut_5.yaml")))
    seeds = [0, 319]
    seq = {s: solve(create("maxcut", cfg, s, 1, verbose=False), cfg, quiet=True, verbose=False) for s in seeds}
    preps = {s: create("maxcut", cfg, s, 1, verbose=False) for s in seeds}  # main thread, global RNG
    out, errs = {}, []

    def run(s):
        try:
            rng.private()
            out[s] = solve(preps[s], cfg, quiet=True, verbose=False)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(e)

    th = [threading.Thread(target=run, args=(s,)) for s in seeds]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for s in seeds:
        for k in ("num_iters", "gap", "feas", "dual_feas", "ranksX", "ranksZ"):
            assert out[s][k] == seq[s][k], (s, k, out[s][k], seq[s][k])
