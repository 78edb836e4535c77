"""Run-to-run spread of bench.py's CPU baseline on one host: the same pinned
oracle workers bench.py starts (PYTHONHASHSEED=0, one core each, whole solves of the YAML seeds),
REPS times back to back, no GPU work in between.
    python tools/cpu_baseline_spread.py [REPS] [--config configs/maxcut_10.yaml]"""
import argparse
import json
import os
import sys

import numpy as np
import yaml

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("reps", type=int, nargs="?", default=2)
ap.add_argument("--config", default=os.path.join(bench.HERE, "configs", "maxcut_10.yaml"))
ap.add_argument("--problem", default="maxcut")
ap.add_argument("--rank", type=int, default=1)
args = ap.parse_args()
seeds = list(yaml.safe_load(open(args.config))["seeds"])
cores = min(len(os.sched_getaffinity(0)), bench.HOST_SHARE)
share = sorted(os.sched_getaffinity(0))[-cores:]
ref = bench.reference_iters(args.config, args.rank, seeds)
meds = []
for rep in range(args.reps):
    procs = bench._spawn_cpu_workers(args, seeds, [1] * len(seeds), 300.0, share[::-1])
    per = bench._release(procs)
    rows = {p["seed"]: (p.get("full_solve_iters"), p.get("full_solve_s_per_iter")) for p in per if p}
    med = float(np.median([v[1] for v in rows.values() if v[1]]))
    meds.append(med)
    print(json.dumps({"rep": rep, "median_s_per_iter": med,
                      "per_seed": {str(s): {"iters": rows[s][0], "reference_iters": ref.get(s),
                                            "s_per_iter": rows[s][1]} for s in rows}}), flush=True)
print(f"medians {['%.4f' % m for m in meds]}  spread (max/min - 1) {max(meds) / min(meds) - 1:.3f}", flush=True)
