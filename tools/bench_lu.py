"""LU (getrf + gecon) and getrs latency: unblocked one-workgroup vs blocked kernels."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402
from tools.bench_linalg import timed  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    st = D._stream()
    print(os.environ.get("TTK_LU_BLOCK_MIN", "default"), "n  getrf+gecon_us  getrs(1 rhs)_us")
    for n in [int(v) for v in os.environ.get("TTK_LU_SIZES", "16,24,32,48,64,80,96,128,200,432").split(",")]:
        A0 = D.from_numpy(rng.standard_normal((n, n)) + n * np.eye(n))
        A = D.empty(n, n)
        piv = torch.empty(n, dtype=torch.int32, device=D.DEV)
        work = D.empty(2 * n + 16)
        rc = ctypes.c_double(0.0)
        b = D.empty(n, 1)

        def f():
            D.copy_(A, A0)
            lib.ttk_lu_sync(st, D._p(A), n, D._p(piv), D._p(work), ctypes.byref(rc))
        t_f = timed(f, reps=5)
        t_s = timed(lambda: lib.ttk_lu_solve(st, D._p(A), n, D._p(piv), D._p(b), 1, 1), reps=10)
        print(f"{n:5d} {t_f:12.1f} {t_s:12.1f}", flush=True)


if __name__ == "__main__":
    main()
