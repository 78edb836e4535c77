#!/usr/bin/env python
"""Headline benchmark: sec / IPM-iteration of the TT-IPM Newton/KKT path on maxcut dim=10 rank=1
(BASELINE.json `metric`, config `configs/maxcut_10.yaml`), seed-sharded over N GPUs.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port P bench.py --gpus N --steps K --warmup W

* Seeds: the config's own list (maxcut_10.yaml: 41, 23, 235, 35, 14) -- nothing else unless
  `--seeds` names them.  A "step" is one full `tt_ipm` solve of one seed per GPU (the reference's
  unit of work, `src/utils.py:245-321`).  Schedule `shard` (default): step i on rank p solves
  seeds[(i*N + p) mod S], so every rank does `--steps` solves (fixed per-GPU work: weak scaling)
  and at N=1 the steps cycle through the config's seeds.  `replica`: every rank solves step i's
  N=1 seed.  Problems are created once per distinct seed on rank 0 and delivered by ONE broadcast
  (RCCL over xGMI with the nccl backend) before the timed region; no collective inside the IPM loop.
* Solves in flight per GPU (`--inflight P`, default 4 at every N, so the 1/2/4/8-GPU series is
  like-for-like): a solve is a chain of small dependent launches that leaves most of the chip idle,
  so each GPU runs P seeds at once.  They run as slot threads (`--threads T`, default 2 per process:
  each thread its own HIP stream, libttk context and NumPy random stream; the launches release the
  GIL) in P/T processes per GPU -- this process plus P/T-1 workers spawned before the GPU is touched
  -- so a node runs at most 16 solve processes (8 GPUs x 2).  All slots warm up, then are released
  together at the start of the timed region.  A step is P solves per GPU: step i, rank p, slot j
  solves seeds[(i*N*P + p*P + j) mod S].
* `solo_median_seed_s_per_iter`: after the timed region (rank 0, N=1) every distinct timed seed is
  solved once more ALONE on the GPU -- SURVEY.md §8(d)'s per-seed latency as the reference runner
  measures it (one solve at a time, `src/utils.py:300-302`); the CPU per-seed comparison uses it.
* Timed region: barrier + device sync on both sides of the K steps, max over ranks.
  `value` = (max-over-ranks wall) / (IPM iterations of all ranks): whole-job s per IPM-iteration.
  `median_seed_s_per_iter` is SURVEY.md §8(d)'s statistic: the median over the distinct seeds of
  each seed's (solve time / iterations).  Seeds the reference runner would call pathological
  (feas or gap > 1e-3, `src/utils.py:67`) are flagged in `per_seed`.
* `roofline` (contraction kernels: the MFMA GEMM `gemm_offs*`, the fused local apply and the Schur
  multi-task apply): an untimed re-solve of rank 0's step-0 seed with every contraction launch
  bracketed by HIP events on its stream.  achieved = ALGORITHMIC contraction FLOPs of that solve
  (NumPy `einsum_path` greedy convention per einsum call plus the chained applies of every local
  KKT operator application; `dev.ALGO`) / summed contraction kernel time; peak =
  78.6 TFLOP/s fp64 matrix.  `device_flops` is what the launched kernels executed.
* `cpu_baseline` (rank 0, N=1 only): the oracle CPU restatement of the reference path (`oracle/`,
  a port) on this host: one single-thread process per core of the host share (16), the timed seeds
  cycled over them, all concurrently, each bounded to the IPM iterations finished within
  `--cpu-cap` seconds.  `value` = median over seeds of the per-seed s/IPM-iter (the statistic of
  SURVEY.md §8(d)); the GPU's per-seed figure over the SAME seeds and iterations (from the timed
  solves' per-iteration timestamps) sits beside it (`gpu_over_cpu`); `throughput` is the concurrent
  run's whole-job s/IPM-iter, the counterpart of this line's `value`.  Then one seed again with all
  the host share's cores as BLAS threads.  The workers are started before this process touches the
  GPU and wait on a pipe until the GPU work is done.
"""
import argparse
import contextlib
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "sec/IPM-iter (AMEn KKT solve), maxcut dim=10 r=1; MFMA util% on core-contract"
FP64_MATRIX_PEAK = 78.6e12  # MI355X spec, FLOP/s
HOST_SHARE = 16  # CPU share of one GPU on the box (nproc shows the whole machine)

# Seeds beyond a config's own list, vetted non-pathological with the oracle in the build container
# (maxcut_12 r=2 lists 5 seeds, the 8-GPU run needs 8).  See DESIGN.md §5.
EXTRA_SEEDS = {"maxcut_12.yaml": [20, 19, 9]}


class _Stop(Exception):
    pass


_CHILDREN = []  # every worker Popen; terminated on any early exit of main()


def _reap_children():
    for p in _CHILDREN:
        if p.poll() is None:
            p.terminate()
    for p in _CHILDREN:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


class _BoundedTrace(list):
    """Trace sink that time-stamps each Newton-system assembly and stops the solve once `cap`
    seconds have passed since the first assembly (after at least one full iteration)."""

    def __init__(self, cap):
        super().__init__()
        self.cap, self.t = cap, []

    def append(self, item):
        self.t.append(time.perf_counter())
        super().append(item)
        if len(self.t) > 1 and self.t[-1] - self.t[0] >= self.cap:
            raise _Stop


def _cpu_worker(problem, cfg_path, seed, rank_tt, cap):
    """Child process: wait for 'go' on stdin, run the oracle on one seed, print one JSON line."""
    import warnings
    from oracle import ipm as OI
    from oracle import problems as OP
    from oracle import tt as OT
    config = yaml.safe_load(open(cfg_path))
    with warnings.catch_warnings(), contextlib.redirect_stdout(sys.stderr):
        warnings.simplefilter("error")
        np.random.seed(seed)
        prob = OP.PROBLEMS[problem](config["dim"], rank_tt, verbose=False)
    if sys.stdin.readline().strip() != "go":  # EOF: the parent is gone -- do not run as an orphan
        sys.exit(3)
    with warnings.catch_warnings(), contextlib.redirect_stdout(sys.stderr):
        warnings.simplefilter("error")
        if len(prob) == 5:
            C, L, b, mask, lag = prob
        else:
            C, L, b, lag_y = prob
            mask, lag = None, {"y": lag_y}
        lag = {k: OT.reshape(v, (4, 4)) for k, v in lag.items()}
        C, b = OT.reshape(C, (4,)), OT.reshape(b, (4,))
        trace = _BoundedTrace(cap if cap > 0 else float("inf"))
        t_start = time.perf_counter()
        try:
            res = OI.tt_ipm(lag, C, L, b, ineq_mask=mask, max_iter=config["max_iter"], verbose=False,
                            gap_tol=float(config["gap_tol"]), op_tol=float(config["op_tol"]),
                            warm_up=config["warm_up"], abs_tol=float(config["abs_tol"]), aho_direction=False,
                            mals_restarts=config["mals_restarts"], max_refinement=config["max_refinement"],
                            lambdaStar=float(config.get("lambdaStar", 1)),
                            lambdaStarIneq=float(config.get("lambdaStarIneq", 1)), trace=trace)
            full = int(res[4]["num_iters"])
            wall = time.perf_counter() - t_start
        except _Stop:
            full, wall = None, None
    n_it = len(trace.t) - 1
    out = {"seed": seed, "iters": n_it, "s_per_iter": (trace.t[n_it] - trace.t[0]) / max(n_it, 1),
           "work_s": trace.t[n_it] - t_start,
           "assembly_t": [t - trace.t[0] for t in trace.t], "threads": os.environ.get("OPENBLAS_NUM_THREADS")}
    if full is not None:
        out.update(full_solve_iters=full, full_solve_s_per_iter=wall / max(full, 1))
    print(json.dumps(out), flush=True)


class _Slots:
    """The solves in flight of one process: one host thread per slot, each with its own HIP stream,
    libttk context (`dev`'s per-thread state) and NumPy random stream (`ttipm_amd.rng`).  Every slot
    thread warms up on its first seed, uploads its problems, then waits for `start()`, solves its
    seeds back to back and records its wall time (its own stream synchronised).  The launches
    themselves release the GIL, so the slots' host work overlaps while their kernels run."""

    def __init__(self, slot_seeds, packed, solve, warmup, device):
        import threading
        self.n = len(slot_seeds)
        self.ready = threading.Barrier(self.n + 1)
        self.go = threading.Event()
        self.out = [None] * self.n
        self.err = []
        self.threads = [threading.Thread(target=self._run, args=(j, sl, packed, solve, warmup, device), daemon=True)
                        for j, sl in enumerate(slot_seeds)]
        for t in self.threads:
            t.start()

    def _run(self, j, seeds, packed, solve, warmup, device):
        import torch
        from ttipm_amd import rng, shard
        preps = None
        try:
            if device is not None:
                torch.cuda.set_device(device)
                # one slot per process: the default stream (measured: two processes on created streams
                # slow each other 2.6x, on their default streams not at all, profiles/r03_inflight_layouts.txt)
                if self.n > 1 or os.environ.get("TTIPM_SLOT_STREAM", "default") != "default":
                    torch.cuda.set_stream(torch.cuda.Stream())
            rng.private()
            for _ in range(warmup):  # untimed: plans, this context's scratch, allocator, code pages
                solve(shard.unpack(*packed[seeds[0]]))
            preps = [shard.unpack(*packed[sd]) for sd in seeds]
            if device is not None:
                torch.cuda.current_stream().synchronize()
        except BaseException as e:  # noqa: BLE001 - re-raised by join()
            self.err.append(e)
        self.ready.wait()
        self.go.wait()
        if preps is None:
            return
        try:
            traces = [[] for _ in seeds]
            t0 = time.perf_counter()
            res = [solve(pr, trace=tr) for pr, tr in zip(preps, traces)]
            if device is not None:
                torch.cuda.current_stream().synchronize()
            elapsed = time.perf_counter() - t0
            for r, tr in zip(res, traces):  # per-iteration stamps (Newton-system assemblies)
                r["assembly_t"] = [e["t"] - tr[0]["t"] for e in tr] if tr else []
            self.out[j] = (elapsed, res)
        except BaseException as e:  # noqa: BLE001
            self.err.append(e)

    def wait_ready(self):
        self.ready.wait()
        if self.err:
            raise RuntimeError(f"bench: a solve slot failed before the timed region: {self.err[0]!r}")

    def start(self):
        self.go.set()

    def join(self):
        for t in self.threads:
            t.join()
        if self.err:
            raise RuntimeError(f"bench: a solve slot failed in the timed region: {self.err[0]!r}")
        return [o[0] for o in self.out], [r for o in self.out for r in o[1]]


def _gpu_worker(args, slot_seeds):
    """Child process (more solves in flight on this rank's GPU): create its seeds' problems, start
    one slot thread per seed list (`_Slots`), print 'ready' once all have warmed up, wait for 'go'
    on stdin, run the solves, print one JSON line with the slots' elapsed wall times and the
    per-seed results."""
    import torch
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    from ttipm_amd import shard
    from ttipm_amd.utils import create
    from ttipm_amd.utils import solve as _solve
    config = yaml.safe_load(open(args.config))
    keep = ("seed", "num_iters", "runtime", "sec_per_iter", "gap", "feas", "dual_feas", "assembly_t")
    with contextlib.redirect_stdout(sys.stderr):  # once, around all slot threads (not thread-safe)
        packed = {s: shard.pack(create(args.problem, config, s, args.rank, verbose=False))
                  for sl in slot_seeds for s in sl}

        def solve(prep, trace=None):
            return _solve(prep, config, quiet=True, verbose=False, trace=trace)

        slots = _Slots(slot_seeds, packed, solve, args.warmup, dev)
        slots.wait_ready()
        print("ready", file=sys.__stdout__, flush=True)
        if sys.stdin.readline().strip() != "go":  # EOF: the parent is gone -- do not run as an orphan
            os._exit(3)
        slots.start()
        elapsed, results = slots.join()
    print(json.dumps({"elapsed": elapsed, "results": [{k: r.get(k) for k in keep} for r in results]}), flush=True)


def _spawn_gpu_workers(args, proc_slots):
    """Started BEFORE this process initialises the GPU; each prints 'ready' once warmed up.
    proc_slots: per worker process, its slots' seed lists."""
    procs = []
    for slots in proc_slots:
        cmd = [sys.executable, os.path.abspath(__file__), "--gpu-worker",
               ";".join(",".join(map(str, sl)) for sl in slots),
               "--problem", args.problem, "--config", args.config, "--rank", str(args.rank),
               "--warmup", str(args.warmup)]
        procs.append(subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=sys.stderr,
                                      text=True))
    _CHILDREN.extend(procs)
    return procs


def _spawn_cpu_workers(args, seeds, threads):
    """Started BEFORE the GPU is initialised (no exec from a GPU process); each blocks on stdin."""
    procs = []
    for s, th in zip(seeds, threads):
        env = dict(os.environ, OPENBLAS_NUM_THREADS=str(th), OMP_NUM_THREADS=str(th), MKL_NUM_THREADS=str(th),
                   CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
        cmd = [sys.executable, os.path.abspath(__file__), "--cpu-worker", str(s), "--problem", args.problem,
               "--config", args.config, "--rank", str(args.rank), "--cpu-cap", str(args.cpu_cap)]
        procs.append(subprocess.Popen(cmd, stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                      stderr=subprocess.DEVNULL, env=env, text=True))
    _CHILDREN.extend(procs)
    return procs


def _release(procs):
    for p in procs:
        p.stdin.write("go\n")
        p.stdin.flush()
    out = []
    for p in procs:
        line = p.stdout.read().strip().splitlines()
        p.wait()
        out.append(json.loads(line[-1]) if line else None)
    return out


def _profiled():
    """True under rocprofv3 (its tool library is preloaded and initialises the GPU before main)."""
    return any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", "")


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def _pmc_traffic():
    """HBM bytes per contraction launch (FETCH_SIZE + WRITE_SIZE, rocprofv3 KB x 1024) from the
    committed PMC passes over the same workload (counters need their own rocprofv3 runs, so they
    cannot be read live here); the newest round's file wins."""
    for name in ("r03_pmc_maxcut10.json", "r02_pmc_maxcut10.json", "r01_pmc_maxcut10.json"):
        try:
            ks = json.load(open(os.path.join(HERE, "profiles", name)))["kernels"]
        except (OSError, KeyError, ValueError):
            continue
        # dispatch-weighted over the gemm_offs_kernel<TS> instantiations
        num = den = 0.0
        for k, e in ks.items():
            base = k.replace("void ", "").split("<")[0].strip()
            if base == "gemm_offs_kernel" and "FETCH_SIZE_KB" in e and "WRITE_SIZE_KB" in e:
                num += (e["FETCH_SIZE_KB"] + e["WRITE_SIZE_KB"]) * e["dispatches"]
                den += e["dispatches"]
        if den:
            return num / den * 1024.0
    return None


DEFAULT_THREADS = 1  # solves in flight per process (slot threads; >1: one created HIP stream each)


def default_inflight(world):
    """Solves in flight per GPU: 4 (one process each, on its default stream) up to 4 GPUs, 2 on 8 GPUs
    (a node runs at most 16 solve processes).  Round-2 process sweep on one MI355X (maxcut_10 whole
    job): 1 -> 0.39, 2 -> 0.20, 4 -> 0.106, 6 -> 0.112 s/IPM-iter: 4 in flight is the knee.  Slot
    threads sharing a process would keep 4 per GPU at N=8, but they need created streams, and
    solves on created streams slow each other down (profiles/r03_inflight_layouts.txt)."""
    return max(1, min(4, DEFAULT_THREADS * (16 // world)))


def make_schedule(config, cfg_name, seeds_arg, steps, world, rank, P, mode):
    """(seeds, per-step seed lists, this rank's per-slot seed lists).  Step i, rank p, slot j
    solves seeds[(i*N*P + p*P + j) mod S] (`shard`) or step i's N=1 seed (`replica`); the config's
    seeds only, plus the vetted EXTRA_SEEDS when a shard step has more solves than seeds."""
    if seeds_arg:
        seeds = [int(s) for s in seeds_arg.split(",")]
    else:
        seeds = list(config["seeds"])
        if mode == "shard" and world * P > len(seeds):
            seeds += [s for s in EXTRA_SEEDS.get(cfg_name, []) if s not in seeds]
    per_step = world * P
    if mode == "shard":
        step_seeds = [seeds[(i * per_step + q) % len(seeds)] for i in range(steps) for q in range(per_step)]
    else:
        step_seeds = [seeds[i % len(seeds)] for i in range(steps) for q in range(per_step)]
    sched = [step_seeds[i * per_step:(i + 1) * per_step] for i in range(steps)]
    slot_seeds = [[sched[i][rank * P + j] for i in range(steps)] for j in range(P)]
    return seeds, sched, slot_seeds


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=os.path.join(HERE, "configs", "maxcut_10.yaml"))
    ap.add_argument("--problem", default=None, help="default: from the config file name")
    ap.add_argument("--rank", type=int, default=1, help="problem rank (create_problem rank)")
    ap.add_argument("--seeds", default=None, help="comma-separated seeds (default: the config's)")
    ap.add_argument("--cpu-cap", type=float, default=60.0, help="seconds of oracle work per seed (0: full solves)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-solo", action="store_true", help="skip the one-solve-at-a-time latency pass")
    ap.add_argument("--schedule", choices=("shard", "replica"), default="shard")
    ap.add_argument("--threads", type=int, default=None,
                    help=f"solves in flight per process (host threads; default {DEFAULT_THREADS})")
    ap.add_argument("--inflight", type=int, default=None,
                    help="solves in flight per GPU (default: default_inflight())")
    ap.add_argument("--cpu-worker", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--gpu-worker", default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.problem is None:
        base = os.path.basename(args.config)
        args.problem = next(p for p in ("maxcut", "corr_clust", "graphm", "max_stable_set") if base.startswith(p))
    if args.cpu_worker is not None:
        return _cpu_worker(args.problem, args.config, args.cpu_worker, args.rank, args.cpu_cap)
    if args.gpu_worker is not None:
        return _gpu_worker(args, [[int(x) for x in sl.split(",")] for sl in args.gpu_worker.split(";")])

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    with open(args.config) as f:
        config = yaml.safe_load(f)
    P = args.inflight if args.inflight else default_inflight(world)
    if _profiled() and (P > 1 or not args.no_cpu_baseline):
        # a profiler's preloaded library has initialised the GPU already: no child processes
        print("bench: under a profiler -> --inflight 1 --no-cpu-baseline", file=sys.stderr)
        P, args.no_cpu_baseline = 1, True
    seeds, sched, slot_seeds = make_schedule(config, os.path.basename(args.config), args.seeds, args.steps, world,
                                             rank, P, args.schedule)
    step_seeds = [s for st in sched for s in st]
    per_step = world * P
    T = max(1, min(args.threads or DEFAULT_THREADS, P))
    if _profiled():
        T = 1
    proc_slots = [slot_seeds[i:i + T] for i in range(0, P, T)]  # this process: proc_slots[0]
    mine_seeds = slot_seeds[0]
    gpu_procs = _spawn_gpu_workers(args, proc_slots[1:])  # before any GPU call

    cpu_seeds = list(dict.fromkeys(s for sl in slot_seeds for s in sl))  # the distinct seeds this (only) rank times
    cpu_procs, allcore_proc = [], []
    do_cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
    cores = min(len(os.sched_getaffinity(0)), HOST_SHARE)
    if do_cpu:  # before any GPU call
        # the host share's cores, one single-thread oracle process each, the timed seeds cycled: the
        # per-seed latency AND the CPU's whole-job throughput come from the same concurrent run
        cyc = [cpu_seeds[i % len(cpu_seeds)] for i in range(max(cores, len(cpu_seeds)))]
        cpu_procs = _spawn_cpu_workers(args, cyc, [1] * len(cyc))
        allcore_proc = _spawn_cpu_workers(args, cpu_seeds[:1], [cores])

    import torch
    import torch.distributed as dist
    if torch.cuda.is_available():
        # one process per GPU; more ranks than GPUs only in rehearsals (TTIPM_BENCH_BACKEND=gloo)
        torch.cuda.set_device(local % torch.cuda.device_count())
    if world > 1:
        backend = os.environ.get("TTIPM_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend)
    from ttipm_amd import dev as D
    from ttipm_amd import shard
    from ttipm_amd._lib import lib
    from ttipm_amd.utils import is_pathological
    from ttipm_amd.utils import solve as _solve

    def solve(prep, trace=None):
        with contextlib.redirect_stdout(sys.stderr):  # stdout carries only the JSON line
            return _solve(prep, config, quiet=True, verbose=False, trace=trace)

    distinct = list(dict.fromkeys(step_seeds))
    with contextlib.redirect_stdout(sys.stderr):
        packed = dict(zip(distinct, shard.broadcast_problems(args.problem, config, distinct, args.rank)))

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    dev_idx = torch.cuda.current_device() if torch.cuda.is_available() else None

    def solve_quiet(prep, trace=None):  # slot threads: stdout is redirected once around them all
        return _solve(prep, config, quiet=True, verbose=False, trace=trace)

    with contextlib.redirect_stdout(sys.stderr):
        sync()
        slots = _Slots(proc_slots[0], packed, solve_quiet, args.warmup, dev_idx)
        slots.wait_ready()
    for p in gpu_procs:  # every worker warmed up and waiting
        line = p.stdout.readline()
        while line and line.strip() != "ready":
            line = p.stdout.readline()
        if not line:
            raise RuntimeError("bench: a GPU worker failed before the timed region")
    barrier()
    sync()
    t0 = time.perf_counter()
    for p in gpu_procs:
        p.stdin.write("go\n")
        p.stdin.flush()
    with contextlib.redirect_stdout(sys.stderr):
        slots.start()
        slot_elapsed, results = slots.join()
    worker_out = []
    for p in gpu_procs:
        line = p.stdout.readline()
        while line and not line.startswith("{"):
            line = p.stdout.readline()
        if p.wait() != 0 or not line:
            raise RuntimeError("bench: a GPU worker failed in the timed region")
        worker_out.append(json.loads(line))
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    slot_elapsed = slot_elapsed + [e for w in worker_out for e in w["elapsed"]]
    results = results + [r for w in worker_out for r in w["results"]]
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
        D.ALGO = {"flops": 0.0, "calls": 0, "by": {}}
        s0, l0 = lib.ttk_sync_count(), lib.ttk_launch_count()
        try:
            rr = solve(shard.unpack(*packed[mine_seeds[0]]))
            sync()
        finally:
            lib.ttk_contract_timing(0)
            algo, D.ALGO = D.ALGO, None
        syncs, all_launches = lib.ttk_sync_count() - s0, lib.ttk_launch_count() - l0
        lib.ttk_contract_stats(st, 1)
        flops, launches, tflops, tl, tms = list(st)
        if tms > 0:
            ach = algo["flops"] / (tms * 1e-3)
            roofline = {"bound": "mfma", "achieved": ach / 1e12, "peak": FP64_MATRIX_PEAK / 1e12,
                        "unit": "TFLOP/s", "frac": ach / FP64_MATRIX_PEAK, "traffic": _pmc_traffic(),
                        "kernel": "contraction kernels: gemm_offs* (fp64 MFMA offset-table GEMM), fused local "
                                  "apply, Schur multi-task apply; traffic = HBM bytes per gemm_offs launch",
                        "seed": mine_seeds[0], "algorithmic_flops_per_solve": algo["flops"],
                        "algorithmic_calls_per_solve": algo["calls"], "device_flops_per_solve": tflops,
                        "launches_per_solve": int(tl), "kernel_ms_per_solve": tms,
                        "all_launches_per_ipm_iter": all_launches / max(rr["num_iters"], 1),
                        "host_syncs_per_ipm_iter": syncs / max(rr["num_iters"], 1),
                        "avg_launch_us": tms * 1e3 / max(tl, 1),
                        "algorithmic_flops_per_launch": algo["flops"] / max(tl, 1),
                        "algorithmic_by_op": dict(sorted(algo["by"].items(), key=lambda kv: -kv[1][1])[:10])}

    # SURVEY.md §8(d)'s per-seed statistic as the reference runner measures it (src/utils.py:300-302:
    # one solve at a time): every distinct timed seed solved once more, alone on the GPU (untimed
    # for `value`; rank 0 at N=1)
    solo = None
    if rank == 0 and world == 1 and not args.no_solo:
        solo = []
        for sd in dict.fromkeys(step_seeds):
            tr = []
            r = solve(shard.unpack(*packed[sd]), trace=tr)
            r["assembly_t"] = [e["t"] - tr[0]["t"] for e in tr] if tr else []
            solo.append(r)
        sync()

    cpu = None
    if do_cpu:
        with contextlib.redirect_stdout(sys.stderr):
            per = _release(cpu_procs)
            allc = _release(allcore_proc)[0]
        gpu_runs, cpu_runs = {}, {}
        for r in (solo or results):  # the GPU's one-at-a-time latency when measured
            gpu_runs.setdefault(r["seed"], []).append(r["assembly_t"])
        for c in per:
            if c is not None and c["iters"] > 0:
                cpu_runs.setdefault(c["seed"], []).append(c["assembly_t"])
        rows = []
        for sd in cpu_runs:  # per seed: the common prefix of IPM iterations of all its runs
            if sd not in gpu_runs:
                continue
            k = min(len(t) - 1 for t in cpu_runs[sd] + gpu_runs[sd])
            if k <= 0:
                continue
            ck = float(np.median([(t[k] - t[0]) / k for t in cpu_runs[sd]]))
            gk = float(np.median([(t[k] - t[0]) / k for t in gpu_runs[sd]]))
            rows.append({"seed": sd, "iters": k, "cpu_runs": len(cpu_runs[sd]), "gpu_runs": len(gpu_runs[sd]),
                         "cpu_s_per_iter": ck, "gpu_s_per_iter": gk, "gpu_over_cpu": gk / ck})
        med = float(np.median([r["cpu_s_per_iter"] for r in rows])) if rows else None
        gmed = float(np.median([r["gpu_s_per_iter"] for r in rows])) if rows else None
        done = [c for c in per if c is not None]
        cpu_iters = sum(c["iters"] for c in done)
        cpu_wall = max((c["work_s"] for c in done), default=0.0)
        cpu = {"value": med, "unit": "s/IPM-iter", "cores": 1, "kind": "port",
               "sample": f"oracle/ CPU restatement of the reference path on {args.problem} dim={config['dim']} "
                         f"rank={args.rank}: {len(done)} single-thread processes at once (the host share's cores), "
                         f"the timed seeds {sorted(cpu_runs)} cycled over them; each process runs its seed's first "
                         f"IPM iterations up to {args.cpu_cap:g} s of work; value = median over seeds of each "
                         f"seed's s/IPM-iter (median over its processes), over the iterations the CPU and GPU "
                         f"runs of that seed have in common; the GPU side is "
                         + ("the one-solve-at-a-time pass (each seed alone on the GPU)" if solo else
                            "the timed in-flight solves"),
               "per_seed": rows,
               "gpu_same_sample_median": gmed,
               "gpu_over_cpu": (gmed / med) if med and gmed else None,
               "gpu_over_cpu_median": float(np.median([r["gpu_over_cpu"] for r in rows])) if rows else None,
               "throughput": {"s_per_iter": cpu_wall / cpu_iters if cpu_iters else None, "processes": len(done),
                              "threads_each": 1, "ipm_iters": cpu_iters, "wall_s": cpu_wall,
                              "note": "whole-job s/IPM-iter of the concurrent CPU run: longest process's work time "
                                      "/ IPM iterations of all processes (the GPU's `value` formula)"},
               "all_cores": None if allc is None else {
                   "seed": allc["seed"], "threads": int(allc["threads"]), "iters": allc["iters"],
                   "cpu_s_per_iter": allc["s_per_iter"]},
               "host": {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "model": _cpu_model()}}

    if rank == 0:
        per_seed, by_seed = [], {}
        for r in all_results:
            per_seed.append({k: r[k] for k in ("seed", "num_iters", "runtime", "sec_per_iter", "gap", "feas",
                                               "dual_feas")})
            per_seed[-1]["pathological"] = bool(is_pathological(r))
            acc = by_seed.setdefault(r["seed"], [0.0, 0])
            acc[0] += r["runtime"]
            acc[1] += r["num_iters"]
        med = float(np.median([t / max(n, 1) for t, n in by_seed.values()]))
        out = {"metric": METRIC, "value": elapsed / max(iters, 1), "unit": "s/IPM-iter", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps,
               "higher_is_better": False, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic: the reference's generators (seeded MT19937 graph TT), problems broadcast "
                       "from rank 0",
               "config": {"workload": f"{args.problem} dim={config['dim']} rank={args.rank} "
                                      f"({os.path.basename(args.config)}), {P} concurrent tt_ipm solves per GPU "
                                      f"per step ({len(proc_slots)} processes x {T} slot threads)",
                          "inflight_per_gpu": P,
                          "seeds": seeds, "seeds_per_step": sched,
                          "parallelism": f"seed-parallel x{world} GPUs x{P} in flight ({args.schedule})",
                          "total_ipm_iters": iters},
               "median_seed_s_per_iter": med,
               "solo_median_seed_s_per_iter": None if not solo else
               float(np.median([r["runtime"] / max(r["num_iters"], 1) for r in solo])),
               "solo_per_seed": None if not solo else
               [{k: r[k] for k in ("seed", "num_iters", "runtime", "sec_per_iter", "gap")} for r in solo],
               "threads_per_process": T,
               "pathological_seeds": sorted({p["seed"] for p in per_seed if p["pathological"]}),
               # library / path knobs set for this run (several change summation order, hence results at
               # rounding level)
               "env_knobs": {k: v for k, v in sorted(os.environ.items()) if k.startswith(("TTK_", "TTIPM_"))},
               "roofline": roofline, "cpu_baseline": cpu,
               "mfma_util_pct": None if roofline is None else 100.0 * roofline["frac"],
               # like-for-like ratios: per-seed latency (the same statistic on both sides) and whole-job
               # throughput (this line's value against the concurrent CPU run's)
               "gpu_over_cpu_per_seed_median": None if cpu is None else cpu["gpu_over_cpu"],
               "gpu_over_cpu_throughput": None if cpu is None or not cpu["throughput"]["s_per_iter"] else
               (elapsed / max(iters, 1)) / cpu["throughput"]["s_per_iter"],
               "per_seed": per_seed}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    finally:
        _reap_children()
