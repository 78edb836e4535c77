"""Two solves of one seed in one process (the first warms plans and allocations); prints the wall time
at which the second starts, for tools/busy_fraction.py's t_from.
    python tools/solve_twice.py maxcut maxcut_10 41 1"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                                       cfg_name + ".yaml")))
t0 = time.time()
r1 = run_and_record(prob, cfg, seed, rank, verbose=False)
t1 = time.time()
r2 = run_and_record(prob, cfg, seed, rank, verbose=False)
t2 = time.time()
print(f"first {t1 - t0:.3f} s, second {t2 - t1:.3f} s ({r2['num_iters']} iterations, "
      f"{(t2 - t1) / r2['num_iters']:.4f} s/iter), second starts at +{t1 - t0:.3f} s", flush=True)
