#!/usr/bin/env python
"""Headline benchmark: sec / IPM-iteration of the TT-IPM Newton/KKT path on maxcut dim=10 rank=1
(BASELINE.json `metric`, config `configs/maxcut_10.yaml`), seed-sharded over N GPUs.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

* A "step" is one full `tt_ipm` solve of one seed per GPU (the reference's unit of work,
  `src/utils.py:245-321`).  Default `--schedule replica`: every rank solves the seed of step i of
  the N=1 run, so per-GPU work is fixed as N grows (weak scaling).  `--schedule shard`: rank p
  solves seeds[i*N + p] (distinct seeds; the makespan is the slowest seed's -- maxcut_10 seed 23
  needs ~6x the work of seed 41).  Problems are created on rank 0 and delivered by ONE RCCL broadcast before
  the timed region (`shard.broadcast_problems`); there is no collective inside the IPM loop.
* Timed region: barrier + device sync on both sides of the K steps, max over ranks.
  value = (max-over-ranks wall) / (IPM iterations of all ranks) -- whole-job s per IPM-iteration.
* `roofline`: the dominant compute kernel is the contraction GEMM (`gemm_offs_kernel`, fp64
  MFMA).  A separate untimed roofline pass re-solves the step-0 seed with every contraction launch
  bracketed by HIP events on its own stream; achieved = algorithmic FLOPs (2*M*N*K per GEMM
  step) / summed kernel time; peak = 78.6 TFLOP/s fp64 matrix (MI355X spec).
* `cpu_baseline` (rank 0, N=1 only): the oracle CPU restatement of the reference path (`oracle/`,
  a port, single BLAS thread) timed on this host over the first few IPM iterations of the same
  seed -- a bounded sample of the same workload.
"""
import argparse
import contextlib
import ctypes
import json
import os
import sys
import time

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "sec/IPM-iter (AMEn KKT solve), maxcut dim=10 r=1; MFMA util% on core-contract"
FP64_MATRIX_PEAK = 78.6e12  # MI355X spec, FLOP/s


def _seed_list(config, n):
    seeds = list(config["seeds"])
    extra = 0
    while len(seeds) < n:  # deterministic extension (SURVEY.md §8(d) maxcut_12 note)
        if extra not in seeds:
            seeds.append(extra)
        extra += 1
    return seeds


class _Stop(Exception):
    pass


class _BoundedTrace(list):
    """Trace sink that time-stamps each Newton-system assembly and stops the solve after `n`."""

    def __init__(self, n):
        super().__init__()
        self.n, self.t = n, []

    def append(self, item):
        self.t.append(time.perf_counter())
        super().append(item)
        if len(self) > self.n:
            raise _Stop


def cpu_baseline(problem, config, seed, rank_tt, iters):
    """Oracle (CPU restatement of the reference path) on the first `iters` IPM iterations."""
    import warnings
    from threadpoolctl import threadpool_limits
    from oracle import ipm as OI
    from oracle import problems as OP
    from oracle import tt as OT
    with threadpool_limits(1), warnings.catch_warnings():
        warnings.simplefilter("error")
        np.random.seed(seed)
        prob = OP.PROBLEMS[problem](config["dim"], rank_tt, verbose=False)
        if len(prob) == 5:
            C, L, b, mask, lag = prob
        else:
            C, L, b, lag_y = prob
            mask, lag = None, {"y": lag_y}
        lag = {k: OT.reshape(v, (4, 4)) for k, v in lag.items()}
        C, b = OT.reshape(C, (4,)), OT.reshape(b, (4,))
        trace = _BoundedTrace(iters if iters > 0 else 10 ** 9)
        t_start = time.perf_counter()
        try:
            res = OI.tt_ipm(lag, C, L, b, ineq_mask=mask, max_iter=config["max_iter"], verbose=False,
                      gap_tol=float(config["gap_tol"]), op_tol=float(config["op_tol"]), warm_up=config["warm_up"],
                      abs_tol=float(config["abs_tol"]), aho_direction=False, mals_restarts=config["mals_restarts"],
                      max_refinement=config["max_refinement"], lambdaStar=float(config.get("lambdaStar", 1)),
                      lambdaStarIneq=float(config.get("lambdaStarIneq", 1)), trace=trace)
            t_end = time.perf_counter()
        except _Stop:
            t_end = None
    if t_end is not None:  # full solve: reference timing (t3 - t2) / num_iters, src/utils.py:300-302
        n_it = int(res[4]["num_iters"])
        val = (t_end - t_start) / max(n_it, 1)
        what = f"full solve, {n_it} IPM iterations, (t3 - t2) / num_iters as src/utils.py:300-302"
    else:
        n_it = len(trace.t) - 1
        val = (trace.t[n_it] - trace.t[0]) / max(n_it, 1)
        what = f"IPM iterations 1..{n_it} (Newton-system assembly to assembly)"
    return {"value": val, "unit": "s/IPM-iter", "cores": 1, "kind": "port",
            "sample": f"{problem} dim={config['dim']} rank={rank_tt} seed {seed}: {what}; oracle/ CPU "
                      f"restatement of the reference path, 1 BLAS thread"}


def _pmc_traffic():
    """HBM bytes per gemm_offs_kernel launch (FETCH_SIZE + WRITE_SIZE, raw rocprofv3 KB x 1024) from
    the committed PMC passes over the same workload (profiles/r01_pmc_maxcut10.json; counters need
    their own rocprofv3 runs, so they cannot be read live here)."""
    path = os.path.join(HERE, "profiles", "r01_pmc_maxcut10.json")
    try:
        k = json.load(open(path))["kernels"]["gemm_offs_kernel"]
        return (k["FETCH_SIZE_KB"] + k["WRITE_SIZE_KB"]) * 1024.0
    except (OSError, KeyError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=os.path.join(HERE, "configs", "maxcut_10.yaml"))
    ap.add_argument("--problem", default="maxcut")
    ap.add_argument("--rank", type=int, default=1, help="problem rank (create_problem rank)")
    ap.add_argument("--cpu-iters", type=int, default=0,
                    help="IPM iterations in the CPU-baseline sample (0 = the full solve of the step-0 seed)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--schedule", choices=("replica", "shard"), default="replica",
                    help="replica: every rank solves the seed of the N=1 step (fixed per-GPU work: weak "
                         "scaling); shard: ranks take distinct seeds of the config (makespan = slowest seed)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if torch.cuda.is_available():
        # one process per GPU; more ranks than GPUs only in rehearsals (TTIPM_BENCH_BACKEND=gloo)
        torch.cuda.set_device(local % torch.cuda.device_count())
    if world > 1:
        backend = os.environ.get("TTIPM_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend)
    from ttipm_amd import shard
    from ttipm_amd._lib import lib
    from ttipm_amd.utils import solve as _solve

    def solve(prep, cfg, quiet=True):
        with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the JSON line
            return _solve(prep, cfg, quiet=quiet, verbose=False)

    with open(args.config) as f:
        config = yaml.safe_load(f)
    if args.schedule == "shard":
        seeds = _seed_list(config, args.steps * world)
        step_seeds = [seeds[(i * world + p) % len(seeds)] for i in range(args.steps) for p in range(world)]
    else:
        seeds = _seed_list(config, args.steps)
        step_seeds = [seeds[i % len(seeds)] for i in range(args.steps) for p in range(world)]
    sched = [step_seeds[i * world:(i + 1) * world] for i in range(args.steps)]
    with contextlib.redirect_stdout(sys.stderr):
        packed = shard.broadcast_problems(args.problem, config, step_seeds, args.rank)
    mine = [packed[i * world + rank] for i in range(args.steps)]

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):  # untimed: same problems as step 0 (plans, allocator, code pages)
        solve(shard.unpack(*mine[0]), config, quiet=True)
    barrier()
    sync()
    t0 = time.perf_counter()
    results = [solve(shard.unpack(*m), config, quiet=True) for m in mine]
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    iters = sum(r["num_iters"] for r in results)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        n = torch.tensor([float(iters)], dtype=torch.float64, device=t.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
        elapsed, iters = float(t.item()), int(n.item())
    all_results = shard.gather_results(results)

    roofline = None
    if not args.no_roofline and rank == 0:
        st = (ctypes.c_double * 5)()
        lib.ttk_contract_stats(st, 1)
        lib.ttk_contract_timing(1)
        solve(shard.unpack(*mine[0]), config, quiet=True)
        sync()
        lib.ttk_contract_timing(0)
        lib.ttk_contract_stats(st, 1)
        flops, launches, tflops, tl, tms = list(st)
        if tms > 0:
            ach = tflops / (tms * 1e-3)
            roofline = {"bound": "mfma", "achieved": ach / 1e12, "peak": FP64_MATRIX_PEAK / 1e12,
                        "unit": "TFLOP/s", "frac": ach / FP64_MATRIX_PEAK, "traffic": _pmc_traffic(),
                        "kernel": "contraction kernels: gemm_offs (fp64 MFMA 16x16x4 offset-table GEMM) + fused "
                                  "local apply + Schur multi-task apply; traffic = per gemm_offs launch",
                        "flops_per_launch": tflops / max(tl, 1), "avg_launch_us": tms * 1e3 / max(tl, 1),
                        "launches_per_solve": int(tl), "kernel_ms_per_solve": tms}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        with contextlib.redirect_stdout(sys.stderr):
            cpu = cpu_baseline(args.problem, config, step_seeds[0], args.rank, args.cpu_iters)

    if rank == 0:
        out = {"metric": METRIC, "value": elapsed / max(iters, 1), "unit": "s/IPM-iter", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
               "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic: reference generators (seeded MT19937 maxcut graph TT), problems broadcast "
                       "from rank 0",
               "config": {"workload": f"{args.problem} dim={config['dim']} rank={args.rank} "
                                      f"({os.path.basename(args.config)}), one tt_ipm solve per GPU per step",
                          "seeds_per_step": sched, "parallelism": f"seed-parallel x{world} ({args.schedule})",
                          "total_ipm_iters": iters},
               "roofline": roofline, "cpu_baseline": cpu,
               "mfma_util_pct": None if roofline is None else 100.0 * roofline["frac"],
               "per_seed": [{k: r[k] for k in ("seed", "num_iters", "runtime", "sec_per_iter", "gap", "feas",
                                               "dual_feas")} for r in all_results]}
        if cpu is not None:
            out["gpu_over_cpu"] = out["value"] / cpu["value"]
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
