"""Whole solves with the step-size eigen-ALS orchestrated natively (_ttkbind.eig_als) and in Python,
alternating in one process after a warm-up solve: per-seed s/IPM-iter of each, and whether the end
points (iterations, gap, feasibility, ranks) are identical to the last digit.
    python tools/ab_native_eig.py maxcut maxcut_10 41,14,23,35,235 [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

import torch  # noqa: E402

from ttipm_amd import tt_eig as E  # noqa: E402
from ttipm_amd import tt_ipm as I  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

EIG_T = [0.0]
AMEN_T = [0.0]


def _timed(f, acc):  # device-synchronised wall time inside the calls of f
    def g(*a, **k):
        torch.cuda.synchronize()
        t = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            torch.cuda.synchronize()
            acc[0] += time.perf_counter() - t
    return g


I.tt_max_generalised_eigen = _timed(I.tt_max_generalised_eigen, EIG_T)
I.tt_restarted_block_amen = _timed(I.tt_restarted_block_amen, AMEN_T)

prob, cfg_name = sys.argv[1], sys.argv[2]
seeds = [int(s) for s in sys.argv[3].split(",")]
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                                       cfg_name + ".yaml")))
run_and_record(prob, cfg, seeds[0], 1, verbose=False)  # warm-up: plans, allocations, constants
keys = ("num_iters", "gap", "feas", "dual_feas", "ranksX")
for seed in seeds:
    for rep in range(reps):
        res = {}
        for native in (True, False):
            E._NATIVE = native
            c0 = dict(E.NATIVE_CALLS)
            EIG_T[0] = AMEN_T[0] = 0.0
            t0 = time.time()
            r = run_and_record(prob, cfg, seed, 1, verbose=False)
            dt = time.time() - t0
            calls = {k: E.NATIVE_CALLS[k] - c0[k] for k in c0}
            res[native] = r
            print(f"seed {seed} rep {rep} {'native' if native else 'python'}: {dt:.3f} s, {r['num_iters']} iters, "
                  f"{dt / r['num_iters']:.4f} s/iter (eigen-ALS {EIG_T[0]:.3f} s, AMEn {AMEN_T[0]:.3f} s), gap {r['gap']:.12e}, eig calls {calls}", flush=True)
        E._NATIVE = True
        same = all(repr(res[True][k]) == repr(res[False][k]) for k in keys)
        print(f"seed {seed} rep {rep}: end points identical: {same}", flush=True)
