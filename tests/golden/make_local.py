"""Reference fixtures for the dense local KKT solves (build container only).

    OPENBLAS_NUM_THREADS=1 PYTHONHASHSEED=0 python tests/golden/make_golden.py local

Runs the reference's own IPM (maxcut_10 seed 41 for `_ipm_local_solver`, src/tt_ipm.py:183-282;
corr_clust_9 seed 764 in fixed mode for `_ipm_local_solver_ineq`, :284-401) with the module-level
local solver wrapped, records the arguments and results of the first local solves, then stops the
run.  From the recorded dense cases it builds the reference's failure cases by perturbing ONE input
block and calling the reference's local solver on it:

* `chol`: the (2,1) operator core negated -> B21 is negative definite, `scipy.linalg.cholesky`
  raises LinAlgError (src/tt_ipm.py:204-207 / :300-303) and the reference falls back to LGMRES;
* `ill` (equality only): the (0,0) block zeroed and the (0,1) core reduced to one large rank-1
  term -> the Schur complement A is 1e-11 I plus a rank-deficient part, `scipy.linalg.solve`
  emits LinAlgWarning (raised: warnings are errors in the reference's IPM, src/tt_ipm.py:16).

Each case stores the inputs (environments, operator cores, aliases / transposes, right-hand-side
environments, previous solution, size_limit, dense_solve), the reference's six return values and
the exception class the reference printed (parsed from its own `⚠️ <Class> in ...` line).
Only data is written (tests/golden/local.npz); no reference source is copied."""
import contextlib
import io
import os
import re
import warnings

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


class _Enough(Exception):
    pass


def _put_case(out, name, args, res, exc):
    XAX_k, A_k, XAX_k1, Xb_k, b_k, Xb_k1, prev, size_limit, dense = args
    for (i, j), v in XAX_k.items():
        if v is not None:
            out[f"{name}/XL{i}{j}"] = np.asarray(v)
    for (i, j), v in XAX_k1.items():
        if v is not None:
            out[f"{name}/XR{i}{j}"] = np.asarray(v)
    keys = list(A_k.keys())
    out[f"{name}/keys"] = np.array(keys, dtype=np.int64)
    for (i, j) in keys:
        out[f"{name}/A{i}{j}"] = np.asarray(A_k[i, j])
    out[f"{name}/transposes"] = np.array([[*k, *v] for k, v in A_k._transposes.items()], dtype=np.int64).reshape(-1, 4)
    out[f"{name}/aliases"] = np.array([[*k, *v] for k, v in A_k._aliases.items()], dtype=np.int64).reshape(-1, 4)
    for i, v in Xb_k.items():
        out[f"{name}/bL{i}"] = np.asarray(v)
    for i, v in Xb_k1.items():
        out[f"{name}/bR{i}"] = np.asarray(v)
    for i in b_k:
        out[f"{name}/b{i}"] = np.asarray(b_k[i])
    out[f"{name}/prev"] = np.asarray(prev)
    out[f"{name}/size_limit"] = np.array(size_limit)
    out[f"{name}/dense_solve"] = np.array(bool(dense))
    sol, res_old, res_min, rhs, nrhs, failed = res
    out[f"{name}/sol"] = np.asarray(sol)
    out[f"{name}/res_old"] = np.array(float(res_old))
    out[f"{name}/res_min"] = np.array(float(res_min))
    out[f"{name}/rhs"] = np.asarray(rhs)
    out[f"{name}/nrhs"] = np.array(float(nrhs))
    out[f"{name}/failed"] = np.array(bool(failed))
    out[f"{name}/exc"] = np.array(exc or "")


def _rebuild_view(rals, A_k, replace):
    """the reference's own TTBlockMatrixView over copies of one core step's operator cores (its
    block_local_product is what the local solver calls), with `replace`d blocks"""
    data = {k: [np.array(A_k[k], copy=True)] for k in A_k.keys()}
    for k, f in replace.items():
        data[k][0] = f(data[k][0])
    return rals.TTBlockMatrixView(data, dict(A_k._aliases), dict(A_k._transposes), 0)


def _call(solver, args):
    buf = io.StringIO()
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        with contextlib.redirect_stdout(buf):
            res = solver(*args)
    m = re.search(r"⚠️ (\w+)", buf.getvalue())
    return res, (m.group(1) if m else None), buf.getvalue()


def _capture(ripm, rops, mod, config, rank, seed, name, want):
    """run the reference IPM until `want(records)` says enough local solves were recorded"""
    recs = []
    orig = getattr(ripm, name)

    def hooked(*args):
        args = list(args) + [True] * (9 - len(args))  # dense_solve default
        res, exc, _ = _call(orig, args)
        snap = ([{k: (None if v is None else np.array(v, copy=True)) for k, v in args[0].items()}, args[1],
                 {k: (None if v is None else np.array(v, copy=True)) for k, v in args[2].items()},
                 {k: np.array(v, copy=True) for k, v in args[3].items()},
                 {k: np.array(args[4][k], copy=True) for k in args[4]},
                 {k: np.array(v, copy=True) for k, v in args[5].items()},
                 np.array(args[6], copy=True), args[7], args[8]])
        snap[1] = _rebuild_view(_rals(), args[1], {})
        recs.append((snap, tuple(np.array(r, copy=True) if isinstance(r, np.ndarray) else r for r in res), exc))
        if want(recs):
            raise _Enough
        return res

    setattr(ripm, name, hooked)
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            np.random.seed(seed)
            prob = mod.create_problem(config["dim"], rank)
            if len(prob) == 5:
                C, L, b, mask, lag = prob
            else:
                C, L, b, lag_y = prob
                mask, lag = None, {"y": lag_y}
            lag = {k: rops.tt_reshape(v, (4, 4)) for k, v in lag.items()}
            try:
                ripm.tt_ipm(lag, rops.tt_reshape(C, (4,)), L, rops.tt_reshape(b, (4,)), ineq_mask=mask,
                            max_iter=config["max_iter"], verbose=False, gap_tol=float(config["gap_tol"]),
                            op_tol=float(config["op_tol"]), warm_up=config["warm_up"],
                            abs_tol=float(config["abs_tol"]), aho_direction=False,
                            mals_restarts=config["mals_restarts"], max_refinement=config["max_refinement"],
                            lambdaStar=float(config.get("lambdaStar", 1)),
                            lambdaStarIneq=float(config.get("lambdaStarIneq", 1)))
            except _Enough:
                pass
    finally:
        setattr(ripm, name, orig)
    return recs, orig


_RALS = []


def _rals():
    return _RALS[0]


def _is_dense(snap):
    prev, size_limit, dense = snap[6], snap[7], snap[8]
    return bool(dense) and np.sqrt(prev.shape[0] * prev.shape[3]) <= size_limit


def main(import_reference):
    import importlib
    rops, rals, ripm = import_reference(True)
    _RALS[:] = [rals]
    out = {}
    # ---- equality: maxcut_10 s41 (src/tt_ipm.py:183-282)
    cfg = yaml.safe_load(open(os.path.join(REF, "configs", "maxcut_10.yaml")))
    mod = importlib.import_module("psd_system.maxcut.maxcut")

    def m_of(r):
        return r[0][6].shape[0] * r[0][6].shape[2] * r[0][6].shape[3]

    def want_eq(recs):
        dense_ok = [r for r in recs if _is_dense(r[0]) and not r[1][5]]
        iters = [r for r in recs if not _is_dense(r[0]) and r[1][1] >= 1e-5]
        return any(m_of(r) >= 256 for r in dense_ok) and len(iters) >= 2

    recs, solver = _capture(ripm, rops, mod, cfg, 1, 41, "_ipm_local_solver", want_eq)
    dense_ok = sorted([r for r in recs if _is_dense(r[0]) and not r[1][5]], key=m_of)
    picks = [dense_ok[0], dense_ok[len(dense_ok) // 2], dense_ok[-1]]
    iters = [r for r in recs if not _is_dense(r[0]) and r[1][1] >= 1e-5][:2]
    names = []
    for i, (snap, res, exc) in enumerate(picks):
        _put_case(out, f"eq_dense{i}", snap, res, exc)
        names.append(f"eq_dense{i}")
    for i, (snap, res, exc) in enumerate(iters):
        _put_case(out, f"eq_iter{i}", snap, res, exc)
        names.append(f"eq_iter{i}")
    base = picks[-1][0]
    # Cholesky failure: B21 negative definite
    snap = list(base)
    snap[1] = _rebuild_view(rals, base[1], {(2, 1): lambda c: -c})
    res, exc, log = _call(solver, snap)
    assert res[5] and exc == "LinAlgError", (exc, log)
    _put_case(out, "eq_chol", snap, res, exc)
    names.append("eq_chol")
    # ill-conditioned Schur complement: B00 = 0 and a rank-1, large B01
    snap = list(base)

    def rank1(c):
        z = np.zeros_like(c)
        z[0, 0, 0, 0] = 1e5
        return z
    snap[1] = _rebuild_view(rals, base[1], {(0, 0): np.zeros_like, (0, 1): rank1})
    res, exc, log = _call(solver, snap)
    assert res[5] and exc == "LinAlgWarning", (exc, log)
    _put_case(out, "eq_ill", snap, res, exc)
    names.append("eq_ill")
    # ---- inequality: corr_clust_9 s764, fixed lgmres_cy.pyx:510 (src/tt_ipm.py:284-401)
    cfg = yaml.safe_load(open(os.path.join(REF, "configs", "corr_clust_9.yaml")))
    mod = importlib.import_module("psd_system.corr_clust.corr_clust")

    def is_dense_ineq(s):
        prev, size_limit, dense = s[6], s[7], s[8]
        return bool(dense) and np.sqrt(prev.shape[0] * prev.shape[3]) <= 0.95 * size_limit

    def want_ineq(recs):
        ok = [r for r in recs if is_dense_ineq(r[0]) and not r[1][5]]
        return any(m_of(r) >= 200 for r in ok)

    recs, solver = _capture(ripm, rops, mod, cfg, 1, 764, "_ipm_local_solver_ineq", want_ineq)
    ok = sorted([r for r in recs if is_dense_ineq(r[0]) and not r[1][5]], key=m_of)
    picks = [ok[0], ok[len(ok) // 2], ok[-1]]
    for i, (snap, res, exc) in enumerate(picks):
        _put_case(out, f"ineq_dense{i}", snap, res, exc)
        names.append(f"ineq_dense{i}")
    iters = sorted([r for r in recs if not is_dense_ineq(r[0])], key=lambda r: -r[1][1])[:1]
    for i, (snap, res, exc) in enumerate(iters):
        _put_case(out, f"ineq_iter{i}", snap, res, exc)
        names.append(f"ineq_iter{i}")
    base = picks[-1][0]
    snap = list(base)
    snap[1] = _rebuild_view(rals, base[1], {(2, 1): lambda c: -c})
    res, exc, log = _call(solver, snap)
    assert res[5] and exc == "LinAlgError", (exc, log)
    _put_case(out, "ineq_chol", snap, res, exc)
    names.append("ineq_chol")
    out["cases"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "local.npz"), **out)
    for n in names:
        print(n, "m =", int(np.prod(out[n + "/prev"].shape)) // out[n + "/prev"].shape[1], "failed", bool(out[n + "/failed"]),
              "exc", str(out[n + "/exc"]) or "-", "res_old %.3e res_min %.3e" % (out[n + "/res_old"], out[n + "/res_min"]))
