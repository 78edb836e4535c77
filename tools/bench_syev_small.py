"""Per-call time of the small extreme-eigenpair kernel (n < 64) -- run once per TTK_SYEV_WAVES8
setting (0: 4 waves; 1: 8 waves, the same symv; bit-identical; the round-6 measurement was taken with
the equivalent TTK_SYEV_SMALL_NT=256 / 512 of the first build):
    TTK_SYEV_WAVES8=0 python tools/bench_syev_small.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402

rng = np.random.default_rng(3)
row = []
for n in (8, 16, 24, 32, 40, 48, 56, 63):
    M = rng.standard_normal((n, n))
    A = D.from_numpy(M + M.T)
    for _ in range(20):
        D.syev_extreme(A)
    torch.cuda.synchronize()
    reps = 200
    t = time.perf_counter()
    for _ in range(reps):
        D.syev_extreme(A)
    torch.cuda.synchronize()
    row.append(f"n={n}: {(time.perf_counter() - t) / reps * 1e6:.1f} us")
print(f"TTK_SYEV_WAVES8={os.environ.get('TTK_SYEV_WAVES8', '1')}: " + ", ".join(row), flush=True)
