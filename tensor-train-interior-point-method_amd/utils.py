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

from . import rng as _rng
from . import tt_ops as T
from .problems import PROBLEMS
from .tt_ipm import IneqStatus, tt_ipm


def _sync():
    """Wait for this thread's launch stream (the whole path runs on it; other host threads' solves
    on other streams are not waited for)."""
    if torch.cuda.is_available():
        torch.cuda.current_stream().synchronize()


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
    _rng.R().set_state(prepared["rng_state"])
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


def save_results_summary(config, cfg_path, rank, results, out_dir="results", args=None):
    """`src/utils.py:210-243`: the same JSON keys (`config_str`, `args_str`, per-seed arrays shaped
    (num_ranks=1, num_seeds), `memory`) plus `sec_per_iter`; file name as the reference builds it
    (`<config>_trackmem_<bool>_seeds_<s1-s2..>_ranks_<rank>.json`)."""
    os.makedirs(out_dir, exist_ok=True)
    seeds = "-".join(str(r["seed"]) for r in results)
    track = bool(getattr(args, "track_mem", False))
    stem = os.path.basename(cfg_path)[:-5] if cfg_path.endswith(".yaml") else os.path.basename(cfg_path)
    name = re.sub(r"[^a-zA-Z0-9_.-]", "_", f"{stem}_trackmem_{track}_seeds_{seeds}_ranks_{'-'.join(str(rank))}.json")
    data = {"config_str": str(config), "args_str": str(vars(args)) if args is not None else "{}",
            "runtimes": [[r["runtime"] for r in results]],
            "problem_creation_times": [[r["creation_time"] for r in results]],
            "num_iters": [[r["num_iters"] for r in results]],
            "feasibility_errors": [[r["feas"] for r in results]],
            "dual_feasibility_errors": [[r["dual_feas"] for r in results]],
            "complementary_slackness": [[r["gap"] for r in results]],
            "ranksX": [[r["ranksX"] for r in results]], "ranksY": [[r["ranksY"] for r in results]],
            "ranksZ": [[r["ranksZ"] for r in results]],
            "ranksT": [[r["ranksT"] for r in results]] if any(any(r["ranksT"]) for r in results) else [],
            "memory": [[r.get("memory", 0.0) for r in results]],
            "sec_per_iter": [[r["sec_per_iter"] for r in results]]}
    path = os.path.join(out_dir, name)
    with open(path, "w") as f:
        json.dump(data, f, indent=2)
    return path


def is_pathological(res):
    """The reference runner's rule (`src/utils.py:67`): feasibility error or slackness > 1e-3."""
    return res["feas"] > 1e-3 or res["gap"] > 1e-3


def _run_tracked(prob, config, seed, rank, track_mem):
    """`run_and_record` with `--track_mem`: the reference records the peak host RSS growth of the
    solve (`memory_profiler`, `src/utils.py:292-296`, MB); here the solve's data lives in HBM, so
    the recorded figure is the peak device allocation growth during the solve (MB)."""
    if not track_mem or not torch.cuda.is_available():
        return run_and_record(prob, config, seed, rank)
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    res = run_and_record(prob, config, seed, rank)
    torch.cuda.synchronize()
    res["memory"] = (torch.cuda.max_memory_allocated() - base) / 2 ** 20
    return res


def run_experiment(problem=None, argv=None):
    """`run_experiment(create_problem_fn)` (`src/utils.py:13-101`): CLI --config/--rank/--track_mem.

    Pathological seeds (`is_pathological`) are replaced as the reference does (`src/utils.py:67-84`):
    a new seed is drawn with `np.random.randint(0, 2**10)` from the global RNG as the previous solve
    left it, skipping used seeds, and the solve is rerun in the same slot.  The reference also
    rewrites the YAML file with the replacement; that happens here only with `--rewrite_config`
    (the seed-sharded multi-GPU path never replaces seeds).  `--no_replace`
    reports the config's seeds as they are."""
    ap = argparse.ArgumentParser(description="TT-IPM on MI355X")
    ap.add_argument("--problem", default=problem, choices=sorted(PROBLEMS))
    ap.add_argument("--config", required=True)
    ap.add_argument("--rank", type=int, default=1)
    ap.add_argument("--track_mem", action="store_true")
    ap.add_argument("--seeds", type=str, default=None, help="comma-separated override of the config seeds")
    ap.add_argument("--no_replace", action="store_true", help="keep pathological seeds (no replacement)")
    ap.add_argument("--rewrite_config", action="store_true", help="write replacement seeds back to the YAML")
    args = ap.parse_args(argv)
    with open(args.config) as f:
        config = yaml.safe_load(f)
    prob = args.problem or next(p for p in PROBLEMS if os.path.basename(args.config).startswith(p))
    if args.seeds:
        config["seeds"] = [int(s) for s in args.seeds.split(",")]
    used = set(config["seeds"])
    results = []
    print(f"\n===== Processing Rank: {args.rank} =====")
    for s_i, seed in enumerate(list(config["seeds"])):
        print(f"Running seed {seed}")
        res = _run_tracked(prob, config, seed, args.rank, args.track_mem)
        while not args.no_replace and is_pathological(res):
            print(f"Seed {res['seed']} is pathological (feasibility error: {res['feas']:.2e}, slackness: "
                  f"{res['gap']:.2e}). Suggesting a new seed.")
            new_seed = np.random.randint(0, 2 ** 10)
            while new_seed in used:
                new_seed = np.random.randint(0, 2 ** 10)
            print(f"New seed suggested: {new_seed}")
            used.add(new_seed)
            config["seeds"][s_i] = int(new_seed)
            if args.rewrite_config:
                with open(args.config, "w") as f:
                    yaml.safe_dump(config, f)
            res = _run_tracked(prob, config, int(new_seed), args.rank, args.track_mem)
            print(f"Rerun with new seed {new_seed} complete. Feasibility error: {res['feas']:.2e}, "
                  f"Slackness: {res['gap']:.2e}")
        results.append(res)
    print_results_summary(config, results)
    return save_results_summary(config, args.config, args.rank, results, args=args)


if __name__ == "__main__":
    run_experiment()
