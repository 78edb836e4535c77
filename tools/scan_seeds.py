"""Diagnostics (GPU): solve a config for a range of seeds on the device and print which end
non-pathological (`src/utils.py:67`: feasibility and gap <= 1e-3).  A diagnostic only: the extra
seeds of configs[4] are chosen from the reference's own runs by a fixed rule (bench.EXTRA_SEEDS,
DESIGN.md section 5), never from device results or timings.

    python tools/scan_seeds.py maxcut maxcut_12 2 7 30"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd.utils import is_pathological, run_and_record  # noqa: E402

prob, cfg_name, rank, lo, hi = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                                       cfg_name + ".yaml")))
for seed in range(lo, hi + 1):
    t = time.perf_counter()
    r = run_and_record(prob, cfg, seed, rank, verbose=False)
    print(json.dumps({"seed": seed, "num_iters": r["num_iters"], "gap": r["gap"], "feas": r["feas"],
                      "pathological": bool(is_pathological(r)), "s": round(time.perf_counter() - t, 1)}),
          flush=True)
