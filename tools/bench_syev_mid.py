"""Per-call time of the extreme eigenpair on the multi-launch path (128 < n <= 513), run once per
TTK_BT_STAGE setting (the env default of TTK_KNOB_BT_STAGE) (1: the finish kernel's back-transform reads its reflectors from LDS blocks staged
by the idle waves; 0: each reflector loaded from global memory one ahead; bit-identical):
    TTK_BT_STAGE=0 python tools/bench_syev_mid.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402

rng = np.random.default_rng(5)
row = []
for n in (144, 192, 256, 300, 352, 448, 512):
    M = rng.standard_normal((n, n))
    A = D.from_numpy(M + M.T)
    for _ in range(5):
        D.syev_extreme(A)
    torch.cuda.synchronize()
    reps = 30
    t = time.perf_counter()
    for _ in range(reps):
        D.syev_extreme(A)
    torch.cuda.synchronize()
    row.append(f"n={n}: {(time.perf_counter() - t) / reps * 1e3:.3f} ms")
print(f"TTK_BT_STAGE={os.environ.get('TTK_BT_STAGE', '1')}: " + ", ".join(row), flush=True)
