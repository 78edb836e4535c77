"""Generate golden vectors from the REFERENCE itself (run in the build container only).

    OPENBLAS_NUM_THREADS=1 python tests/golden/make_golden.py [runs|prims|all] [config...]

* imports `/root/reference/src/*` and `/root/reference/psd_system/*` as they lie, with the
  reference's Cython kernels compiled from source into `oracle/_ref` (`oracle/build_ref.py`);
* third-party packages absent from the image are replaced by `tests/golden/refshim/`
  (opt_einsum -> numpy.einsum greedy; petsc4py KSPLGMRES -> oracle/petsc_lgmres.py restatement;
  scikit-sparse / memory_profiler -> unused stubs);
* the reference's `IneqMatVecWrapper.matvec` returns a memoryview (`cy_src/lgmres_cy.pyx:510`);
  "fixed" runs load the variant built by oracle/build_ref.py with that one line corrected
  (SURVEY.md §0.5), "shipped" runs load the module as written; each run is its own process;
* writes `tests/golden/runs.json` (per-seed final metrics + per-Newton-system trace) and
  `tests/golden/prims.npz` (primitive-level input/output pairs).

Only data is written; no reference source is copied.  The fixtures are consumed by tests/.
"""
import json
import os
import sys
import time

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("OMP_NUM_THREADS", "1")

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
REF = "/root/reference"
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import yaml  # noqa: E402


def patch_svd(kind):
    """SVD-algorithm twins: the reference's scipy.linalg.svd calls (default gesdd, or the explicit
    lapack_driver='gesvd' of the rounding / eigen code) on another LAPACK algorithm -- 'jacobi':
    dgejsv (one-sided Jacobi, high relative accuracy, the algorithm class of the device SVD),
    'gesvd' / 'swap': the other bidiagonalisation driver.  Rounding-level variation of the
    reference's own computation, like the thread and hash-seed twins."""
    import scipy.linalg as sla
    from scipy.linalg import lapack
    orig = sla.svd

    def svd(a, *args, **kw):
        if kind == "jacobi":
            a = np.asarray(a, dtype=float)
            if a.shape[0] < a.shape[1]:
                u, s, vt = svd(a.T)
                return vt.T, s, u.T
            sva, u, v, work, _, info = lapack.dgejsv(np.array(a, order="F"), joba=1, jobu=0, jobv=0)
            if info == 0:
                return u, sva * (work[0] / work[1]), v.T
            kw.pop("lapack_driver", None)
        elif kind == "swap":
            kw["lapack_driver"] = "gesdd" if kw.get("lapack_driver", "gesdd") == "gesvd" else "gesvd"
        elif "lapack_driver" not in kw:
            kw["lapack_driver"] = kind
        return orig(a, *args, **kw)
    sla.svd = svd


def _import_reference(fixed_ineq=True):
    from oracle.build_ref import build
    build()
    if os.environ.get("GOLDEN_SVD"):
        patch_svd(os.environ["GOLDEN_SVD"])
    cy = os.path.join(REPO, "oracle", "_ref", "fixed") if fixed_ineq else os.path.join(REPO, "oracle", "_ref")
    sys.path[:0] = [os.path.join(HERE, "refshim"), cy, REF]
    import src.tt_ops as rops  # noqa
    import src.tt_als as rals  # noqa
    import src.tt_ipm as ripm  # noqa
    import warnings
    warnings.simplefilter("default")  # tt_ipm sets "error" at import; re-enabled around runs
    return rops, rals, ripm


PROBLEM_MOD = {"maxcut": "psd_system.maxcut.maxcut", "corr_clust": "psd_system.corr_clust.corr_clust",
               "graphm": "psd_system.graphm.graphm", "max_stable_set": "psd_system.max_stable_set.max_stable_set"}


class _Bounded(Exception):
    """Raised by the trace hook once `max_assemblies` Newton systems have been assembled."""


def run_reference(problem, cfg_name, seed, rank, fixed_ineq=True, max_assemblies=0):
    """Mirror of `src/utils.py:245-321` (run_and_record) with a per-Newton-system trace hook.

    `max_assemblies > 0` gives a BOUNDED trace (configs whose full reference run does not fit the
    build container's budget): the run stops right after that many Newton-system assemblies and
    records, besides the trace, every AMEn KKT solve (`tt_restarted_block_amen`: residual, solution
    ranks) and every step-size pair (`_tt_get_step_sizes`) made before the stop."""
    import importlib
    import warnings
    rops, rals, ripm = _import_reference(fixed_ineq)
    with open(os.path.join(REF, "configs", cfg_name + ".yaml")) as f:
        config = yaml.safe_load(f)
    mod = importlib.import_module(PROBLEM_MOD[problem])
    trace = []
    orig = ripm.tt_infeasible_newton_system

    def hooked(lhs, obj, X, Y, Z, Tt, L, Ladj, b, mask, status):
        out = orig(lhs, obj, X, Y, Z, Tt, L, Ladj, b, mask, status)
        st = out[2]
        trace.append({"mu": float(st.mu), "primal_error": float(st.primal_error),
                      "dual_error": float(st.dual_error), "centrality_error": float(st.centrality_error),
                      "sigma": float(st.sigma), "ranksX": rops.tt_ranks(X), "ranksZ": rops.tt_ranks(Z),
                      "ranksY": rops.tt_ranks(Y), "is_last_iter": bool(st.is_last_iter)})
        return out

    amen, steps = [], []
    orig_amen, orig_steps = ripm.tt_restarted_block_amen, ripm._tt_get_step_sizes

    def hooked_amen(*a, **k):
        t0 = time.time()
        sol, res = orig_amen(*a, **k)
        amen.append({"res": float(res), "ranks": [int(c.shape[-1]) for c in sol[:-1]],
                     "block_core": [int(i) for i, c in enumerate(sol) if c.ndim == 4][:1],
                     "seconds": time.time() - t0})
        return sol, res

    def hooked_steps(*a, **k):
        xs, zs = orig_steps(*a, **k)
        steps.append([float(xs), float(zs)])
        return xs, zs

    def bounded(*a, **k):
        out = hooked(*a, **k)
        if max_assemblies and len(trace) >= max_assemblies:
            raise _Bounded
        return out

    ripm.tt_infeasible_newton_system = bounded
    ripm.tt_restarted_block_amen = hooked_amen
    ripm._tt_get_step_sizes = hooked_steps
    if max_assemblies:
        return _run_bounded(ripm, rops, mod, config, problem, cfg_name, seed, rank, fixed_ineq, max_assemblies,
                            trace, amen, steps)
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        np.random.seed(seed)
        prob = mod.create_problem(config["dim"], rank)
        if len(prob) == 5:
            C, L, b, mask, lag = prob
        else:
            C, L, b, lag_y = prob
            mask = None
            lag = {"y": lag_y}
        lag = {k: rops.tt_reshape(v, (4, 4)) for k, v in lag.items()}
        C = rops.tt_reshape(C, (4,))
        b = rops.tt_reshape(b, (4,))
        t2 = time.time()
        X, Y, Tt, Z, info = ripm.tt_ipm(lag, C, L, b, ineq_mask=mask, max_iter=config["max_iter"], verbose=False,
                                        gap_tol=float(config["gap_tol"]), op_tol=float(config["op_tol"]),
                                        warm_up=config["warm_up"], abs_tol=float(config["abs_tol"]),
                                        aho_direction=False, mals_restarts=config["mals_restarts"],
                                        max_refinement=config["max_refinement"],
                                        lambdaStar=float(config.get("lambdaStar", 1)),
                                        lambdaStarIneq=float(config.get("lambdaStarIneq", 1)))
        t3 = time.time()
        gap = abs(rops.tt_inner_prod(X, Z))
        pr = rops.tt_rank_reduce(rops.tt_sub(rops.tt_fast_matrix_vec_mul(L, rops.tt_reshape(X, (4,))), b), eps=1e-12)
        feas = rops.tt_inner_prod(pr, pr)
        dr = rops.tt_rank_reduce(rops.tt_sub(rops.tt_fast_matrix_vec_mul(rops.tt_transpose(L), rops.tt_reshape(Y, (4,)), eps=1e-12),
                                             rops.tt_rank_reduce(rops.tt_add(rops.tt_reshape(Z, (4,)), C), eps=1e-12)), eps=1e-12)
        if info["status"].ineq_status is ripm.IneqStatus.ACTIVE:
            dr = rops.tt_rank_reduce(rops.tt_sub(dr, rops.tt_reshape(Tt, (4,))), eps=1e-12)
        dfeas = rops.tt_inner_prod(dr, dr)
    ripm.tt_infeasible_newton_system = orig
    ripm.tt_restarted_block_amen, ripm._tt_get_step_sizes = orig_amen, orig_steps
    return {"problem": problem, "config": cfg_name, "seed": seed, "rank": rank, "fixed_ineq": fixed_ineq,
            "num_iters": int(info["num_iters"]), "runtime": t3 - t2,
            "sec_per_iter": (t3 - t2) / max(1, int(info["num_iters"])), "gap": float(gap), "feas": float(feas),
            "hash_seed": os.environ.get("PYTHONHASHSEED"), "svd": os.environ.get("GOLDEN_SVD") or "scipy default",
            "petsc_kernels": os.environ.get("GOLDEN_PETSC_KERNELS") == "1",
            "dual_feas": float(dfeas), "ranksX": info["ranksX"], "ranksY": info["ranksY"],
            "ranksZ": info["ranksZ"], "trace": trace, "blas_threads": os.environ.get("OPENBLAS_NUM_THREADS")}


def _run_bounded(ripm, rops, mod, config, problem, cfg_name, seed, rank, fixed_ineq, n, trace, amen, steps):
    import warnings
    t2 = time.time()
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        np.random.seed(seed)
        prob = mod.create_problem(config["dim"], rank)
        if len(prob) == 5:
            C, L, b, mask, lag = prob
        else:
            C, L, b, lag_y = prob
            mask = None
            lag = {"y": lag_y}
        lag = {k: rops.tt_reshape(v, (4, 4)) for k, v in lag.items()}
        C = rops.tt_reshape(C, (4,))
        b = rops.tt_reshape(b, (4,))
        try:
            ripm.tt_ipm(lag, C, L, b, ineq_mask=mask, max_iter=config["max_iter"], verbose=False,
                        gap_tol=float(config["gap_tol"]), op_tol=float(config["op_tol"]),
                        warm_up=config["warm_up"], abs_tol=float(config["abs_tol"]), aho_direction=False,
                        mals_restarts=config["mals_restarts"], max_refinement=config["max_refinement"],
                        lambdaStar=float(config.get("lambdaStar", 1)),
                        lambdaStarIneq=float(config.get("lambdaStarIneq", 1)))
            stopped = False
        except _Bounded:
            stopped = True
    return {"problem": problem, "config": cfg_name, "seed": seed, "rank": rank, "fixed_ineq": fixed_ineq,
            "bounded": n, "stopped": stopped, "seconds": time.time() - t2, "trace": trace, "amen": amen,
            "steps": steps, "blas_threads": os.environ.get("OPENBLAS_NUM_THREADS")}


# (problem, config, seed, rank, fixed_ineq, max_assemblies): max_assemblies > 0 = bounded trace
RUNS = [
    ("maxcut", "maxcut_5", 0, 1, True, 0),
    ("maxcut", "maxcut_5", 319, 1, True, 0),
    ("maxcut", "maxcut_10", 41, 1, True, 0),
    ("maxcut", "maxcut_10", 23, 1, True, 0),
    ("maxcut", "maxcut_10", 235, 1, True, 0),
    ("maxcut", "maxcut_10", 35, 1, True, 0),
    ("maxcut", "maxcut_10", 14, 1, True, 0),
    ("corr_clust", "corr_clust_9", 764, 1, True, 0),
    ("corr_clust", "corr_clust_9", 764, 1, False, 0),
    ("graphm", "graphm_3", 256, 2, True, 2),
    ("graphm", "graphm_3", 256, 2, True, 0),
    ("maxcut", "maxcut_12", 80, 2, True, 0),
    # the bench's extra maxcut_12 seeds (configs[4] needs 8 distinct seeds for 8 ranks): vetted as
    # non-pathological by these reference runs (src/utils.py:67-84)
    ("maxcut", "maxcut_12", 0, 2, True, 0),  # pathological in the reference (29 iterations, gap 2.1e-2)
    ("maxcut", "maxcut_12", 1, 2, True, 0),  # 16 iterations, gap 9.2e-4 (hash twins: bounded_twins.json)
    ("maxcut", "maxcut_12", 2, 2, True, 0),  # pathological in the reference (29 iterations, gap 4.3e-2)
    ("maxcut", "maxcut_12", 3, 2, True, 0),  # pathological in the reference (14 iterations, gap 1.3e-2)
    ("maxcut", "maxcut_12", 4, 2, True, 0),  # pathological in the reference (13 iterations, gap 0.38)
    ("maxcut", "maxcut_12", 5, 2, True, 0),  # pathological in the reference (10 iterations, gap 4.7)
    ("maxcut", "maxcut_12", 6, 2, True, 0),  # pathological in the reference (29 iterations, gap 2.1e-2)
    ("maxcut", "maxcut_12", 7, 2, True, 0),  # pathological in the reference (24 iterations, gap 5.3)
    ("maxcut", "maxcut_12", 8, 2, True, 0),  # pathological in the reference (29 iterations, gap 6.0e-3)
    ("maxcut", "maxcut_12", 9, 2, True, 0),
    ("maxcut", "maxcut_12", 10, 2, True, 0),  # pathological in the reference (29 iterations, gap 2.2e-2)
    ("maxcut", "maxcut_12", 11, 2, True, 0),  # 14 iterations, gap 2.6e-4 (hash twins: bounded_twins.json)
    ("maxcut", "maxcut_12", 13, 2, True, 0),  # pathological in the reference (29 iterations, gap 0.66)
    ("maxcut", "maxcut_12", 16, 2, True, 0),  # pathological in the reference (12 iterations, gap 0.17)
    ("maxcut", "maxcut_12", 18, 2, True, 0),  # pathological in the reference (17 iterations, gap 1.16e-3)
    ("maxcut", "maxcut_12", 19, 2, True, 0),
    ("maxcut", "maxcut_12", 20, 2, True, 0),
    # the rest of configs/maxcut_12.yaml's seeds: bounded traces (3 Newton systems each, every AMEn
    # solve and step pair before them) -- a full 1-thread reference run is ~35 min per seed
    ("maxcut", "maxcut_12", 45, 2, True, 3),
    ("maxcut", "maxcut_12", 23, 2, True, 3),
    ("maxcut", "maxcut_12", 53, 2, True, 3),
    ("maxcut", "maxcut_12", 12, 2, True, 3),
    # ... and their full runs (round 5: the device's end points on these seeds need a reference)
    ("maxcut", "maxcut_12", 45, 2, True, 0),
    ("maxcut", "maxcut_12", 23, 2, True, 0),
    ("maxcut", "maxcut_12", 53, 2, True, 0),
    ("maxcut", "maxcut_12", 12, 2, True, 0),
]


THREADS = int(os.environ.get("GOLDEN_THREADS", "1"))  # >1: the thread-spread runs (key suffix _t<N>)
# != 0: the summation-order twins (key suffix _h<N>): opt_einsum orders tensordot axes by frozenset
# iteration, so PYTHONHASHSEED picks among equally valid summation orders of every contraction --
# the reference's own rounding-level noise, at every problem size (1 vs 8 BLAS threads perturbs
# nothing below BLAS's threading thresholds)
HASH = int(os.environ.get("GOLDEN_HASH", "0"))
SVD = os.environ.get("GOLDEN_SVD", "")  # SVD-algorithm twins (key suffix _j<hash> for 'jacobi', patch_svd)
# PETSc-reduction twins (key suffix _p<hash>): the LGMRES restatement with PETSc's Seq reduction
# kernels (dnrm2, index-order VecMDot, grouped VecMAXPY; oracle/petsc_lgmres.py PETSC_KERNELS)
PETSC = os.environ.get("GOLDEN_PETSC_KERNELS") == "1"


def run_key(cfg, rank, seed, fixed, nmax):
    return f"{cfg}_r{rank}_s{seed}" + ("" if fixed else "_shipped") + (f"_b{nmax}" if nmax else "") + \
        (f"_t{THREADS}" if THREADS > 1 else "") + \
        (f"_p{HASH}" if PETSC else
         (f"_j{HASH}" if SVD == "jacobi" else (f"_{SVD}{HASH}" if SVD else (f"_h{HASH}" if HASH else ""))))


def make_runs(only=None, jobs=1):
    """Each run in its own process (1 BLAS thread, PYTHONHASHSEED=0: opt_einsum's tensordot axis order
    follows frozenset iteration, so the hash seed pins the summation order); `jobs` at a time."""
    import subprocess
    todo = []
    for prob, cfg, seed, rank, fixed, nmax in RUNS:
        key = run_key(cfg, rank, seed, fixed, nmax)
        if only and cfg not in only and key not in only:
            continue
        todo.append((key, [sys.executable, __file__, "one", prob, cfg, str(seed), str(rank), str(int(fixed)),
                           os.path.join("/tmp", f"golden_{key}.json"), str(nmax)]))
    env = dict(os.environ, PYTHONHASHSEED=str(HASH), OPENBLAS_NUM_THREADS=str(THREADS), OMP_NUM_THREADS=str(THREADS))
    running = []
    while todo or running:
        while todo and len(running) < jobs:
            key, cmd = todo.pop(0)
            print("running reference", key, flush=True)
            running.append((key, cmd[-2], subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL)))
        key, tmp, p = running.pop(0)
        if p.wait() != 0:
            print(key, "FAILED", flush=True)
            continue
        merge(key, tmp)


def merge(key, tmp, store="runs.json"):
    """add one finished run's JSON (`one` mode output) to runs.json (or `store`) under `key`"""
    import fcntl
    path = os.path.join(HERE, store)
    res = json.load(open(tmp))
    print(key, {k: res.get(k) for k in ("num_iters", "gap", "feas", "dual_feas", "sec_per_iter")}, flush=True)
    with open(path + ".lock", "w") as lk:  # several make_runs invocations may merge at once
        fcntl.flock(lk, fcntl.LOCK_EX)
        out = json.load(open(path)) if os.path.exists(path) else {}
        out[key] = res
        with open(path + ".tmp", "w") as f:
            json.dump(out, f, indent=1)
        os.replace(path + ".tmp", path)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        _, _, prob, cfg, seed, rank, fixed, tmp = sys.argv[:8]
        nmax = int(sys.argv[8]) if len(sys.argv) > 8 else 0
        with open(tmp, "w") as f:
            json.dump(run_reference(prob, cfg, int(seed), int(rank), bool(int(fixed)), nmax), f)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "merge":  # merge KEY TMP: a run finished outside make_runs
        merge(sys.argv[2], sys.argv[3])
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "merge_twin":  # merge_twin KEY TMP: a bounded hash twin
        merge(sys.argv[2], sys.argv[3], "bounded_twins.json")
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "local":  # dense local KKT solve fixtures (a6 / a7)
        from tests.golden import make_local
        make_local.main(_import_reference)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "step":  # step-size eigen-ALS fixtures (a19)
        from tests.golden import make_step
        make_step.main(_import_reference)
        sys.exit(0)
    if len(sys.argv) < 2 or sys.argv[1] not in ("runs", "prims", "all"):
        # no default: a bare invocation must not start regenerating (and rewriting) runs.json
        sys.exit("usage: make_golden.py runs|prims|all [KEY ...] [-jN] | one PROB CFG SEED RANK FIXED OUT [NMAX]"
                 " | merge KEY TMP | local")
    what = sys.argv[1]
    rest = [a for a in sys.argv[2:] if not a.startswith("-j")]
    jobs = max([int(a[2:]) for a in sys.argv[2:] if a.startswith("-j")] or [1])
    if what in ("runs", "all"):
        make_runs(rest or None, jobs)
    if what in ("prims", "all"):
        from tests.golden import make_prims
        make_prims.main(_import_reference)
