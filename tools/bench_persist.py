"""Per-call wall time of the one-launch forms against the per-step launches they replace (same
arithmetic): the multi-workgroup Jacobi SVD with one launch per sweep (TTK_KNOB_SVD_SWEEP_ONE) or per
round, and the multi-workgroup tridiagonalisation of the extreme eigenpair with every step in one
launch (TTK_KNOB_TRI_PERSIST) or one launch per step.  Alternating off / on / off / on.
    python tools/bench_persist.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import _lib  # noqa: E402
from ttipm_amd import dev as D  # noqa: E402

rng = np.random.default_rng(1)


def timed(knob, fn, reps=5):
    row = []
    for v in (0, 1, 0, 1):
        _lib.lib.ttk_ctx_set_knob(None, knob, v, None)
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        row.append((time.perf_counter() - t) / reps * 1e3)
    _lib.lib.ttk_ctx_set_knob(None, knob, 1, None)
    return row


for (m, n) in [(120, 100), (150, 120), (200, 130), (260, 255), (400, 130), (600, 400)]:
    A = D.from_numpy(rng.standard_normal((m, n)))
    row = timed(_lib.KNOB_SVD_SWEEP_ONE, lambda: D.svd(A))
    print(f"svd {m}x{n}: per round {row[0]:.3f} / {row[2]:.3f} ms, per sweep {row[1]:.3f} / {row[3]:.3f} ms", flush=True)
for n in (129, 144, 192, 256, 300, 352, 512):
    M = rng.standard_normal((n, n))
    A = D.from_numpy(M + M.T)
    row = timed(_lib.KNOB_TRI_PERSIST, lambda: D.syev_extreme(A))
    print(f"syev_extreme n={n}: per step {row[0]:.3f} / {row[2]:.3f} ms, one launch {row[1]:.3f} / {row[3]:.3f} ms",
          flush=True)
D.check_handoffs()
