"""Repeated solves of one seed in one process (after one warm-up): per-solve s/IPM-iter, for A/B
timing of switches (env vars) with less box-to-box noise than single runs.
    python tools/time_solves.py maxcut maxcut_10 41 1 [reps]"""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd.utils import create, solve  # noqa: E402

prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 4
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", cfg_name + ".yaml")))
out = []
for i in range(reps + 1):
    prep = create(prob, cfg, seed, rank, verbose=False)
    t = time.perf_counter()
    r = solve(prep, cfg, quiet=True, verbose=False)
    dt = time.perf_counter() - t
    if i:
        out.append(dt / r["num_iters"])
print(os.environ.get("TTIPM_TAG", ""), "median s/iter %.4f" % statistics.median(out), ["%.4f" % v for v in out],
      "gap", r["gap"], flush=True)
