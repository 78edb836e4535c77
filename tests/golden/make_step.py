"""Reference fixtures for the step-size eigen-ALS (build container only).

    OPENBLAS_NUM_THREADS=1 PYTHONHASHSEED=0 python tests/golden/make_golden.py step

Runs the reference's own IPM (`src/tt_ipm.py:901-1099`) on maxcut_10 seeds 14 and 41 with
`tt_max_generalised_eigen` (`src/tt_als.py:1132-1283`, reached through `_tt_get_step_sizes`,
`src/tt_ipm.py:700-727`) and its two-site local solve `_step_size_local_solve` (`:931-1038`)
wrapped, and records for every eigen-ALS call of the first `NMAX` Newton systems:

* the whole call: operator TT (X or Z), direction TT (Delta X or Delta Z), warm start x0, the global
  MT19937 state before the call (the ALS draws its kick vectors from it), the step size and the
  solution TT it returned;
* every local solve inside it: the two cores, the eight environment / operator-core inputs, the step
  size, size_limit / trunc_tol / eps / max_rank / bwd, the MT19937 state before it, and the two
  returned cores, step size and old residual.

maxcut_10 s14's assembly-5 dual step is where the reference's unmodified runs take zs = 0.5019 and
the device 0.4057: this isolates that call the way `local.npz` isolates the KKT local
solves.  Only data is written (tests/golden/step.npz); no reference source is copied."""
import os

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
NMAX = {14: 7, 41: 3}  # Newton systems whose step pairs are recorded


class _Enough(Exception):
    pass


def _state():
    s = np.random.get_state()
    return s[1].copy(), int(s[2]), int(s[3]), float(s[4])


def _run(ripm, rals, rops, seed, calls):
    import warnings
    cfg = yaml.safe_load(open(os.path.join(REF, "configs", "maxcut_10.yaml")))
    import importlib
    mod = importlib.import_module("psd_system.maxcut.maxcut")
    orig_eig, orig_loc, orig_nwt = ripm.tt_max_generalised_eigen, rals._step_size_local_solve, \
        ripm.tt_infeasible_newton_system
    n_asm = [0]
    cur = [None]

    def nwt(*a, **k):
        if n_asm[0] >= NMAX[seed]:
            raise _Enough
        n_asm[0] += 1
        return orig_nwt(*a, **k)

    def eig(A, Delta, x0=None, **k):
        rec = {"assembly": n_asm[0] - 1, "A": [c.copy() for c in A], "Delta": [c.copy() for c in Delta],
               "x0": None if x0 is None else [c.copy() for c in x0], "rng": _state(), "local": []}
        cur[0] = rec
        step, x = orig_eig(A, Delta, x0=x0, **k)
        rec["step"] = float(step)
        rec["x"] = [c.copy() for c in x]
        calls.append(rec)
        cur[0] = None
        return step, x

    def loc(*a, **k):
        st = _state()
        out = orig_loc(*a, **k)
        a = a + tuple(k[n] for n in LOCAL_ARGS[len(a):] if n in k)
        if cur[0] is not None:
            cur[0]["local"].append({"args": [np.array(v, copy=True) if isinstance(v, np.ndarray) else v for v in a],
                                    "rng": st, "out": [np.array(o, copy=True) if isinstance(o, np.ndarray) else o
                                                       for o in out]})
        return out

    ripm.tt_max_generalised_eigen, rals._step_size_local_solve, ripm.tt_infeasible_newton_system = eig, loc, nwt
    try:
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            np.random.seed(seed)
            C, L, b, lag_y = mod.create_problem(cfg["dim"], 1)
            lag = {"y": rops.tt_reshape(lag_y, (4, 4))}
            try:
                ripm.tt_ipm(lag, rops.tt_reshape(C, (4,)), L, rops.tt_reshape(b, (4,)), ineq_mask=None,
                            max_iter=cfg["max_iter"], verbose=False, gap_tol=float(cfg["gap_tol"]),
                            op_tol=float(cfg["op_tol"]), warm_up=cfg["warm_up"], abs_tol=float(cfg["abs_tol"]),
                            aho_direction=False, mals_restarts=cfg["mals_restarts"],
                            max_refinement=cfg["max_refinement"], lambdaStar=float(cfg.get("lambdaStar", 1)),
                            lambdaStarIneq=float(cfg.get("lambdaStarIneq", 1)))
            except _Enough:
                pass
    finally:
        ripm.tt_max_generalised_eigen, rals._step_size_local_solve, ripm.tt_infeasible_newton_system = \
            orig_eig, orig_loc, orig_nwt


LOCAL_ARGS = ("p1", "p2", "XAX_k", "A_k", "A_kp1", "XAX_k2", "XDX_k", "D_k", "D_kp1", "XDX_k2", "step",
              "size_limit", "trunc_tol", "eps", "max_rank", "bwd")


def _put_tt(out, name, tt):
    if tt is None:
        return
    out[name + "/n"] = np.array(len(tt))
    for i, c in enumerate(tt):
        out[f"{name}/{i}"] = np.asarray(c)


def _put_rng(out, name, st):
    out[name + "/key"], out[name + "/pos"], out[name + "/g"], out[name + "/c"] = \
        st[0], np.array(st[1]), np.array(st[2]), np.array(st[3])


def _put_call(out, name, rec, with_local):
    _put_tt(out, name + "/A", rec["A"])
    _put_tt(out, name + "/Delta", rec["Delta"])
    _put_tt(out, name + "/x0", rec["x0"])
    _put_tt(out, name + "/x", rec["x"])
    _put_rng(out, name + "/rng", rec["rng"])
    out[name + "/step"] = np.array(rec["step"])
    out[name + "/assembly"] = np.array(rec["assembly"])
    out[name + "/nlocal"] = np.array(len(rec["local"]))
    if not with_local:
        return
    for j, lc in enumerate(rec["local"]):
        p = f"{name}/l{j}"
        for k, v in zip(LOCAL_ARGS, lc["args"]):
            out[f"{p}/{k}"] = np.asarray(v)
        _put_rng(out, p + "/rng", lc["rng"])
        s1, s2, step, res = lc["out"]
        out[p + "/s1"], out[p + "/s2"] = np.asarray(s1), np.asarray(s2)
        out[p + "/step_out"], out[p + "/res"] = np.array(float(step)), np.array(float(res))


def main(import_reference):
    rops, rals, ripm = import_reference(True)
    out, names = {}, []
    for seed in (14, 41):
        calls = []
        _run(ripm, rals, rops, seed, calls)
        for i, rec in enumerate(calls):
            print(f"s{seed} call {i} assembly {rec['assembly']} step {rec['step']:.10e} local solves {len(rec['local'])}",
                  flush=True)
        if seed == 14:  # the assembly-5 step pair (x then z) with every local solve; the earlier calls whole
            keep = [i for i, r in enumerate(calls) if r["assembly"] in (4, 5)]
        else:  # s41, the path-stable headline seed: its first step pairs with every local solve
            keep = [i for i, r in enumerate(calls) if r["assembly"] in (0, 1)]
        for i in keep:
            name = f"s{seed}_c{i}"
            _put_call(out, name, calls[i], with_local=True)
            names.append(name)
    out["cases"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "step.npz"), **out)
    print("wrote", names, flush=True)
