"""Experiment runner -- drop-in for `src/utils.py` (`run_experiment`, `run_and_record`,
summary printing and the JSON results file; SURVEY.md §5 "Metrics / logging").

    python -m ttipm_amd.utils --problem maxcut --config configs/maxcut_10.yaml --rank 1

Timing follows the reference exactly: runtime = t3 - t2 around `tt_ipm` (`src/utils.py:272-302`);
sec/IPM-iteration = runtime / num_iters.  Extra keys: `sec_per_iter`, `trace`."""
import argparse
import json
import os
import re
import time

import numpy as np
import torch
import yaml

from . import tt_ops as T
from .problems import PROBLEMS
from .tt_ipm import IneqStatus, tt_ipm


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def create(problem, config, seed, rank, verbose=None):
    """Problem creation half of `run_and_record` (`src/utils.py:258-270`): seeds the global NumPy
    RNG, builds the problem on the device and returns it with the RNG state the IPM continues
    from (the IPM's own random draws follow creation in the same stream)."""
    verbose = config.get("verbose", False) if verbose is None else verbose
    np.random.seed(seed)
    _sync()
    t1 = time.time()
    prob = PROBLEMS[problem](config["dim"], rank, verbose=verbose)
    if len(prob) == 5:
        C, L, b, mask, lag = prob
    else:
        C, L, b, lag_y = prob
        mask = None
        lag = {"y": lag_y}
    lag = {k: T.tt_reshape(v, (4, 4)) for k, v in lag.items()}
    C = T.tt_reshape(C, (4,))
    b = T.tt_reshape(b, (4,))
    _sync()
    return {"seed": seed, "C": C, "L": L, "b": b, "mask": mask, "lag": lag,
            "rng_state": np.random.get_state(), "creation_time": time.time() - t1}


def solve(prepared, config, trace=None, verbose=None, iter_callback=None, quiet=False):
    """Timed half of `run_and_record` (`src/utils.py:272-321`): `tt_ipm` between t2 and t3, then
    the recorded gap / primal / dual feasibility."""
    verbose = config.get("verbose", False) if verbose is None else verbose
    C, L, b, mask, lag = prepared["C"], prepared["L"], prepared["b"], prepared["mask"], prepared["lag"]
    np.random.set_state(prepared["rng_state"])
    _sync()
    t2 = time.time()
    X, Y, Tt, Z, info = tt_ipm(lag, C, L, b, ineq_mask=mask, max_iter=config["max_iter"], verbose=verbose,
                               gap_tol=float(config["gap_tol"]), op_tol=float(config["op_tol"]),
                               warm_up=config["warm_up"], abs_tol=float(config["abs_tol"]), aho_direction=False,
                               mals_restarts=config["mals_restarts"], max_refinement=config["max_refinement"],
                               lambdaStar=float(config.get("lambdaStar", 1)),
                               lambdaStarIneq=float(config.get("lambdaStarIneq", 1)), trace=trace,
                               iter_callback=iter_callback)
    _sync()
    t3 = time.time()
    gap = abs(T.tt_inner_prod(X, Z))
    pr = T.tt_rank_reduce(T.tt_sub(T.tt_fast_matrix_vec_mul(L, T.tt_reshape(X, (4,))), b), eps=1e-12)
    feas = T.tt_inner_prod(pr, pr)
    dr = T.tt_rank_reduce(T.tt_sub(T.tt_fast_matrix_vec_mul(T.tt_transpose(L), T.tt_reshape(Y, (4,)), eps=1e-12),
                                   T.tt_rank_reduce(T.tt_add(T.tt_reshape(Z, (4,)), C), eps=1e-12)), eps=1e-12)
    if info["status"].ineq_status is IneqStatus.ACTIVE:
        dr = T.tt_rank_reduce(T.tt_sub(dr, T.tt_reshape(Tt, (4,))), eps=1e-12)
    dfeas = T.tt_inner_prod(dr, dr)
    n_it = int(info["num_iters"])
    out = {"seed": prepared["seed"], "creation_time": prepared["creation_time"], "runtime": t3 - t2,
           "num_iters": n_it, "sec_per_iter": (t3 - t2) / max(n_it, 1), "gap": float(gap), "feas": float(feas),
           "dual_feas": float(dfeas), "ranksX": info["ranksX"], "ranksY": info["ranksY"], "ranksZ": info["ranksZ"],
           "ranksT": info["ranksT"]}
    if not quiet:
        print(f"Convergence after {n_it} iterations. Compl Slackness: {gap:.4e}. Feasibility error: {feas:.4e}. "
              f"Dual Feasibility error: {dfeas:.4e}.")
        print(f"Convergence in {t3 - t2:.2f}s ({out['sec_per_iter']:.3f} s/iter).", flush=True)
    return out


def run_and_record(problem, config, seed, rank, trace=None, verbose=None, iter_callback=None):
    """`run_and_record` (`src/utils.py:245-321`) for one seed; returns a dict of the recorded values."""
    return solve(create(problem, config, seed, rank, verbose=verbose), config, trace=trace, verbose=verbose,
                 iter_callback=iter_callback)


def print_results_summary(config, results):
    """`src/utils.py:118-206` (condensed)."""
    rt = np.array([r["runtime"] for r in results])
    it = np.array([r["num_iters"] for r in results])
    spi = np.array([r["sec_per_iter"] for r in results])
    print("\n" + "=" * 80)
    print(f"{'FINAL RESULTS SUMMARY':^80}")
    print("=" * 80)
    print(f"  {'Solution Time (s)':<28} | {f'{rt.mean():.3f} ± {rt.std():.3f}':>25}")
    print(f"  {'Runtime Median (s)':<28} | {f'{np.median(rt):.3f}':>25}")
    print(f"  {'sec / IPM-iter (median)':<28} | {f'{np.median(spi):.4f}':>25}")
    print(f"  {'Iterations':<28} | {f'{it.mean():.1f} ± {it.std():.1f}':>25}")
    for key, name in (("feas", "Feasibility Error"), ("dual_feas", "Dual Feasibility Error"), ("gap", "Duality Gap")):
        v = np.array([r[key] for r in results])
        print(f"  {name:<28} | {f'{v.mean():.2e} ± {v.std():.2e}':>25}")
    print("=" * 80)


def save_results_summary(config, cfg_path, rank, results, out_dir="results"):
    """`src/utils.py:210-243` JSON keys (+ sec_per_iter)."""
    os.makedirs(out_dir, exist_ok=True)
    seeds = "-".join(str(r["seed"]) for r in results)
    name = re.sub(r"[^a-zA-Z0-9_.-]", "_", f"{os.path.basename(cfg_path)[:-5]}_seeds_{seeds}_ranks_{rank}.json")
    data = {"config_str": str(config), "runtimes": [[r["runtime"] for r in results]],
            "problem_creation_times": [[r["creation_time"] for r in results]],
            "num_iters": [[r["num_iters"] for r in results]],
            "feasibility_errors": [[r["feas"] for r in results]],
            "dual_feasibility_errors": [[r["dual_feas"] for r in results]],
            "complementary_slackness": [[r["gap"] for r in results]],
            "ranksX": [[r["ranksX"] for r in results]], "ranksY": [[r["ranksY"] for r in results]],
            "ranksZ": [[r["ranksZ"] for r in results]], "ranksT": [[r["ranksT"] for r in results]],
            "sec_per_iter": [[r["sec_per_iter"] for r in results]]}
    path = os.path.join(out_dir, name)
    with open(path, "w") as f:
        json.dump(data, f, indent=2)
    return path


def run_experiment(problem=None, argv=None):
    """`run_experiment(create_problem_fn)` (`src/utils.py:13-101`): CLI --config/--rank."""
    ap = argparse.ArgumentParser(description="TT-IPM on MI355X")
    ap.add_argument("--problem", default=problem, choices=sorted(PROBLEMS))
    ap.add_argument("--config", required=True)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--track_mem", action="store_true")
    ap.add_argument("--seeds", type=str, default=None, help="comma-separated override of the config seeds")
    args = ap.parse_args(argv)
    with open(args.config) as f:
        config = yaml.safe_load(f)
    prob = args.problem or next(p for p in PROBLEMS if os.path.basename(args.config).startswith(p))
    seeds = [int(s) for s in args.seeds.split(",")] if args.seeds else config["seeds"]
    results = []
    for seed in seeds:
        print(f"Running seed {seed}")
        results.append(run_and_record(prob, config, seed, args.rank))
    print_results_summary(config, results)
    return save_results_summary(config, args.config, args.rank, results)


if __name__ == "__main__":
    run_experiment()
