"""Decision trace of one solve: every local KKT solve (local shape, dense gate, res_old, res_min,
failure flag, whether the previous solution was kept, ||sol||), every AMEn call (residual, ranks),
every step-size pair and every Newton-system assembly, in call order -- the discrete choices the
reference's control flow takes, so two runs can be aligned event by event.

    python tools/decision_trace.py ref maxcut maxcut_10 14 1 [max_assemblies] > ref.jsonl  (build
        container: the REFERENCE itself, imported as tests/golden/make_golden.py does)
    python tools/decision_trace.py dev maxcut maxcut_10 14 1 [max_assemblies] > dev.jsonl  (GPU box)
    python tools/decision_trace.py oracle maxcut maxcut_10 14 1 [max_assemblies]  (the CPU restatement)
    python tools/decision_trace.py diff ref.jsonl dev.jsonl
    DT_RANKS=1 (oracle / dev): also every AMEn truncation rank scan (r0, chosen r, limit, ratios)

Hooks wrap the module-level names the reference's tt_ipm looks up at call time
(`_ipm_local_solver(_ineq)`, `tt_restarted_block_amen`, `_tt_get_step_sizes`,
`tt_infeasible_newton_system`; src/tt_ipm.py:958-981, 589, 666, 700, 1031) and the same names of
ttipm_amd.tt_ipm."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402


REF_NAMES = ("_ipm_local_solver", "_ipm_local_solver_ineq", "tt_restarted_block_amen", "_tt_get_step_sizes",
             "tt_infeasible_newton_system")
ORACLE_NAMES = ("local_solver", "local_solver_ineq", "restarted_block_amen", "step_sizes", "newton_system")


def install(mod, norm, ranks, ev, names=REF_NAMES):
    """wrap mod's hot-path names; norm(t) -> float, ranks(tt) -> list"""
    for name in names[:2]:
        f = getattr(mod, name)

        def ls(*a, _f=f, **k):
            out = _f(*a, **k)
            sol, res_old, res_min, rhs, nrhs, dsf = out
            prev = a[6]
            ev.append({"e": "local", "shape": [int(s) for s in prev.shape], "dense_arg": bool(a[8] if len(a) > 8
                                                                                            else k.get("dense_solve", True)),
                       "res_old": float(res_old), "res_min": float(res_min), "nrhs": float(nrhs), "dsf": bool(dsf),
                       "kept_prev": sol is prev, "sol": norm(sol)})
            return out
        setattr(mod, name, ls)
    amen = getattr(mod, names[2])

    def am(*a, **k):
        ev.append({"e": "amen_begin", "restriction": int(k.get("rank_restriction") or 0), "inner_m": int(k.get("inner_m") or 0)})
        x, res = amen(*a, **k)
        ev.append({"e": "amen", "res": float(res), "ranks": ranks(x)})
        return x, res
    setattr(mod, names[2], am)
    steps = getattr(mod, names[3])

    def stp(*a, **k):
        xs, zs = steps(*a, **k)
        ev.append({"e": "steps", "xs": float(xs), "zs": float(zs)})
        return xs, zs
    setattr(mod, names[3], stp)
    newton = getattr(mod, names[4])

    def nw(*a, **k):
        out = newton(*a, **k)
        st = out[2]
        ev.append({"e": "assembly", "mu": float(st.mu), "primal": float(st.primal_error),
                   "dual": float(st.dual_error), "centrality": float(st.centrality_error), "sigma": float(st.sigma)})
        return out
    setattr(mod, names[4], nw)


def run_ref(problem, cfg, seed, rank, nmax):
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden as MG
    rops, rals, ripm = MG._import_reference(True)
    if os.environ.get("REF_SVD_DRIVER"):  # twin: the reference's default-driver (gesdd) SVDs on another driver
        import scipy.linalg as sla_mod
        orig_svd, drv = sla_mod.svd, os.environ["REF_SVD_DRIVER"]

        from scipy.linalg import lapack as _lp

        def svd(a, *args, **kw):
            if drv == "jacobi":  # LAPACK dgejsv (one-sided Jacobi, high relative accuracy)
                a = np.asarray(a, dtype=float)
                if a.shape[0] < a.shape[1]:
                    u, s_, vt = svd(a.T)
                    return vt.T, s_, u.T
                sva, u, v, work, _, info = _lp.dgejsv(np.array(a, order="F"), joba=1, jobu=0, jobv=0)
                if info == 0:
                    return u, sva * (work[0] / work[1]), v.T
                kw.pop("lapack_driver", None)
            if drv == "swap":  # every call on the other LAPACK driver (gesdd <-> gesvd)
                kw["lapack_driver"] = "gesdd" if kw.get("lapack_driver", "gesdd") == "gesvd" else "gesvd"
            elif "lapack_driver" not in kw:
                kw["lapack_driver"] = drv
            return orig_svd(a, *args, **kw)
        sla_mod.svd = svd
    ev = []
    install(ripm, lambda t: float(np.linalg.norm(t)), lambda x: [int(c.shape[-1]) for c in x[:-1]], ev)
    MG.run_reference(problem, cfg, seed, rank, True, nmax)
    return ev


def run_oracle(problem, cfg_name, seed, rank, nmax):
    """the CPU restatement (oracle/), same hooks and bound"""
    import warnings
    import yaml
    from oracle import ipm as OI
    from oracle import problems as OP
    from oracle import tt as OT
    ev = []
    install(OI, lambda t: float(np.linalg.norm(t)), lambda x: [int(c.shape[-1]) for c in x[:-1]], ev, ORACLE_NAMES)
    if os.environ.get("DT_RANKS"):  # also every AMEn truncation rank scan (oracle/als.py RANK_TRACE)
        from oracle import als as OA_
        OA_.RANK_TRACE = ev
    if os.environ.get("ORACLE_JACOBI_SVD"):  # experiment: LAPACK dgejsv (Jacobi, relative accuracy) SVDs
        import scipy.linalg as sla_mod
        from scipy.linalg import lapack
        from oracle import als as OA
        orig_svd = sla_mod.svd

        def jsvd(a, full_matrices=False, **kw):
            a = np.asarray(a, dtype=float)
            if a.shape[0] < a.shape[1]:
                u, s_, vt = jsvd(a.T)
                return vt.T, s_, u.T
            sva, u, v, work, _, info = lapack.dgejsv(np.array(a, order="F"), joba=1, jobu=0, jobv=0)
            if info != 0:
                return orig_svd(a, full_matrices=False)
            if os.environ.get("ORACLE_JACOBI_SIGNS") == "lapack":  # experiment: LAPACK's singular-vector signs
                ul, _, _ = orig_svd(a, full_matrices=False, lapack_driver="gesvd")
                sg = np.sign(np.sum(u * ul, axis=0))
                sg[sg == 0] = 1.0
                u, v = u * sg, v * sg
            return u, sva * (work[0] / work[1]), v.T

        class _S:  # scipy.linalg facade for oracle/als.py only
            def __getattr__(self, k):
                return jsvd if k == "svd" else getattr(sla_mod, k)
        which = os.environ["ORACLE_JACOBI_SVD"]
        if which == "all":
            sla_mod.svd = jsvd
        else:  # comma list of oracle modules whose SVDs go to dgejsv
            import importlib
            for mname in which.split(","):
                importlib.import_module("oracle." + mname).sla = _S()
    if os.environ.get("ORACLE_KRON_ZIPUP") == "1":  # experiment: the device's zip-up
        from oracle import tt as OTT
        from oracle import als as OA2

        def kron_round(cores, eps):
            return OTT.rank_reduce(cores, eps) if len(cores) > 1 and eps > 0 else cores

        def fmv(mat, vec, eps=1e-18):
            return kron_round([np.einsum("amnA,rnR->armAR", a, x).reshape(a.shape[0] * x.shape[0], a.shape[1],
                                                                            a.shape[3] * x.shape[2])
                               for a, x in zip(mat, vec)], eps)

        def fmm(m1, m2, eps=1e-18):
            return kron_round([np.einsum("amkA,bknB->abmnAB", a, b).reshape(a.shape[0] * b.shape[0], a.shape[1],
                                                                             b.shape[2], a.shape[3] * b.shape[3])
                               for a, b in zip(m1, m2)], eps)

        def fh(t1, t2, eps=1e-18):
            if t1[0].ndim == 4 and t2[0].ndim == 4:
                cs = [np.einsum("aijA,bijB->abijAB", a, b).reshape(a.shape[0] * b.shape[0], a.shape[1], a.shape[2],
                                                                   a.shape[3] * b.shape[3]) for a, b in zip(t1, t2)]
            else:
                cs = [np.einsum("aiA,biB->abiAB", a, b).reshape(a.shape[0] * b.shape[0], a.shape[1],
                                                                a.shape[2] * b.shape[2]) for a, b in zip(t1, t2)]
            return kron_round(cs, eps)
        for mod in (OTT, OI, OA2):
            for name, f in (("fast_matrix_vec_mul", fmv), ("fast_mat_mat_mul", fmm), ("fast_hadamard", fh)):
                if hasattr(mod, name):
                    setattr(mod, name, f)
    if os.environ.get("ORACLE_EXACT_EIG") == "1":  # experiment: exact dense eigenpairs instead of ARPACK
        import scipy.linalg as sla
        import scipy.sparse.linalg as spla
        from oracle import eig as OE
        orig = spla.eigsh

        def exact_min(M, eps, m, v0):
            w, V = np.linalg.eigh(M.toarray())
            return w[:1], V[:, :1].copy()

        def eigsh(A, k=6, M=None, which="LM", **kw):
            if M is not None and which == "LA":
                w, V = sla.eigh(-(-A).toarray(), M.toarray())
                return w[-1:], V[:, -1:].copy()
            return orig(A, k=k, M=M, which=which, **kw)
        OE._eigsh_min_with_polish = exact_min
        OE.spla.eigsh = eigsh
    config = yaml.safe_load(open(os.path.join(ROOT, "configs", cfg_name + ".yaml")))

    class Stop(Exception):
        pass
    inner = OI.newton_system

    def bounded(*a, **k):
        out = inner(*a, **k)
        if nmax and sum(1 for e in ev if e["e"] == "assembly") >= nmax:
            raise Stop
        return out
    OI.newton_system = bounded
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        np.random.seed(seed)
        prob = OP.PROBLEMS[problem](config["dim"], rank, verbose=False)
        if len(prob) == 5:
            C, L, b, mask, lag = prob
        else:
            C, L, b, lag_y = prob
            mask, lag = None, {"y": lag_y}
        lag = {k: OT.reshape(v, (4, 4)) for k, v in lag.items()}
        C, b = OT.reshape(C, (4,)), OT.reshape(b, (4,))
        try:
            OI.tt_ipm(lag, C, L, b, ineq_mask=mask, max_iter=config["max_iter"], verbose=False,
                      gap_tol=float(config["gap_tol"]), op_tol=float(config["op_tol"]),
                      warm_up=config["warm_up"], abs_tol=float(config["abs_tol"]), aho_direction=False,
                      mals_restarts=config["mals_restarts"], max_refinement=config["max_refinement"],
                      lambdaStar=float(config.get("lambdaStar", 1)),
                      lambdaStarIneq=float(config.get("lambdaStarIneq", 1)))
        except Stop:
            pass
    return ev


def run_dev(problem, cfg_name, seed, rank, nmax):
    import torch
    import yaml
    torch.cuda.set_device(0)
    from ttipm_amd import dev as D
    from ttipm_amd import tt_ipm
    from ttipm_amd.utils import run_and_record
    ev = []
    install(tt_ipm, lambda t: float(D.norm(t)), lambda x: [int(c.shape[-1]) for c in x[:-1]], ev)
    if os.environ.get("DT_RANKS"):  # also every AMEn truncation rank scan (tt_als.RANK_TRACE)
        from ttipm_amd import tt_als
        tt_als.RANK_TRACE = ev
    cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", cfg_name + ".yaml")))

    class Stop(Exception):
        pass
    if nmax:
        inner = tt_ipm.tt_infeasible_newton_system

        def bounded(*a, **k):
            out = inner(*a, **k)
            if sum(1 for e in ev if e["e"] == "assembly") >= nmax:
                raise Stop
            return out
        tt_ipm.tt_infeasible_newton_system = bounded
    try:
        run_and_record(problem, cfg, seed, rank, verbose=False)
    except Stop:
        pass
    return ev


KEYS = {"local": ("res_old", "res_min", "nrhs", "sol"), "amen": ("res",), "steps": ("xs", "zs"),
        "assembly": ("mu", "primal", "dual", "centrality", "sigma")}
DISCRETE = {"local": ("shape", "dense_arg", "dsf", "kept_prev"), "amen": ("ranks",), "amen_begin": ("restriction",)}


def diff(a_path, b_path, tol=1e-6):
    A = [json.loads(s) for s in open(a_path) if s.startswith("{")]
    B = [json.loads(s) for s in open(b_path) if s.startswith("{")]
    n_asm = 0
    worst = 0.0
    for i, (a, b) in enumerate(zip(A, B)):
        if a["e"] == "assembly":
            n_asm += 1
        if a["e"] != b["e"]:
            print(f"event {i}: kind differs {a['e']} / {b['e']} (after {n_asm} assemblies)")
            return
        for k in DISCRETE.get(a["e"], ()):
            if a.get(k) != b.get(k):
                print(f"event {i} ({a['e']}, after {n_asm} assemblies): {k} differs: {a.get(k)} / {b.get(k)}")
                for j in range(max(0, i - 4), min(len(A), i + 3)):
                    print("  A", j, A[j])
                    print("  B", j, B[j] if j < len(B) else None)
                return
        for k in KEYS.get(a["e"], ()):
            # residuals near round-off (|r| ~ 1e-10 and below) are noise: absolute floor 1e-12
            floor = 1e-12 if k.startswith("res") else 0.0
            rel = abs(a[k] - b[k]) / max(abs(a[k]), 1e-300) if abs(a[k] - b[k]) > floor else 0.0
            worst = max(worst, rel)
            if rel > tol:
                print(f"event {i} ({a['e']}, after {n_asm} assemblies): {k} rel {rel:.3e}: {a[k]!r} / {b[k]!r}"
                      f"  (worst before: {worst:.2e})")
                for j in range(max(0, i - 4), min(len(A), i + 3)):
                    print("  A", j, A[j])
                    print("  B", j, B[j] if j < len(B) else None)
                return
    print(f"no departure beyond {tol:g} over {min(len(A), len(B))} events (worst {worst:.2e})")


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "diff":
        diff(sys.argv[2], sys.argv[3], float(sys.argv[4]) if len(sys.argv) > 4 else 1e-6)
        sys.exit(0)
    prob, cfg, seed, rank = sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    nmax = int(sys.argv[6]) if len(sys.argv) > 6 else 0
    import contextlib
    with contextlib.redirect_stdout(sys.stderr):
        ev = {"ref": run_ref, "oracle": run_oracle, "dev": run_dev}[mode](prob, cfg, seed, rank, nmax)
    for e in ev:
        print(json.dumps(e))
