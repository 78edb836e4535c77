"""Kernel time of the one-workgroup Householder QR (ttk_qr) at the TT cores' shapes, HIP events on
the launch stream (run with TTK_QR_NARROW=0 / 1 to compare the 1024-thread and the narrow launch)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402
from tools.bench_linalg import timed  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    st = D._stream()
    print("QR narrow" if os.environ.get("TTK_QR_NARROW", "1") != "0" else "QR 1024 threads")
    for m, n in [(10, 5), (24, 6), (16, 4), (8, 2), (4, 5), (48, 12), (56, 14), (128, 8), (16, 12), (64, 40)]:
        A = D.from_numpy(rng.standard_normal((m, n)))
        k = min(m, n)
        Q, R, w = D.empty(m, k), D.empty(k, n), D.empty(int(lib.ttk_qr_work(m, n)))
        t = timed(lambda: lib.ttk_qr(st, D._p(A), m, n, D._p(Q), D._p(R), D._p(w)), reps=200)
        print(f"  qr {m:4d}x{n:<4d} {t:8.2f} us", flush=True)


if __name__ == "__main__":
    main()
