"""Schur-reduced KKT matvec (ttk_schur_apply, cy_src/lgmres_cy.pyx:297-327) latency per operator
size: random operator blocks of maxcut-sized ranks, N back-to-back applies timed with HIP events on
the launch stream.  With a -DTTK_VALU_PROFILE build (TTK_LIB_PATH=...) it also prints the per-row
phase split of these applies only.

    python tools/bench_schur.py [reps]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd import tt_ipm  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402


def op_for(rng, r, s, R, S):
    keys = tt_ipm.MatVecWrapper.keys
    L = {k: D.from_numpy(rng.standard_normal((r, s, r))) for k in keys}
    A = {k: D.from_numpy(rng.standard_normal((s, 4, 4, S))) for k in keys}
    Rr = {k: D.from_numpy(rng.standard_normal((R, S, R))) for k in keys}
    inv = D.from_numpy(rng.uniform(0.5, 2.0, (r, 4, R)))
    return tt_ipm.MatVecWrapper(L, A, Rr, inv, (r, 4, R))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    rng = np.random.default_rng(0)
    prof = (ctypes.c_ulonglong * 8)()
    for r, s, R, S in [(4, 3, 4, 3), (8, 6, 8, 6), (10, 8, 10, 8), (13, 10, 13, 10), (13, 10, 26, 10)]:
        op = op_for(rng, r, s, R, S)
        m = op.m
        v = D.from_numpy(rng.standard_normal(2 * m))
        out = D.empty(2 * m)
        for _ in range(10):
            op.matvec_into(v, out)
        torch.cuda.synchronize()
        lib.ttk_mfma_profile(prof, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            op.matvec_into(v, out)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        lib.ttk_mfma_profile(prof, 0)
        rows = max(prof[7], 1)
        ph = ""
        if prof[7]:
            ph = " | per row (us): staging %.2f s1 %.2f s2 %.2f s3 %.2f; waits %.2f us x %d/matvec" % (
                prof[0] / 100 / rows, prof[1] / 100 / rows, prof[2] / 100 / rows, prof[3] / 100 / rows,
                prof[4] / 100 / max(prof[5], 1), prof[5] // reps)
        print(f"r={r:2d} s={s:2d} R={R:2d} S={S:2d} m={m:5d}: {us:7.2f} us per matvec, "
              f"{prof[7] // reps if prof[7] else 0} rows{ph}", flush=True)


if __name__ == "__main__":
    main()
