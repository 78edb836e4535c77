"""Latency of the one-workgroup SVD on the path's small unfoldings, with phase split."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402
from tools.bench_linalg import counters, timed  # noqa: E402


def main():
    rng = np.random.default_rng(0)
    st = D._stream()
    print("m x n   kernel_us  sweeps  phases_us(qrcp, jacobi, vectors, out)")
    for m, n in [(2, 1), (4, 2), (4, 4), (8, 4), (8, 6), (10, 2), (2, 5), (10, 10), (12, 6), (12, 12), (8, 10),
                 (16, 12), (20, 24), (40, 46)]:
        A = D.from_numpy(rng.standard_normal((m, n)) @ np.diag(0.5 ** np.arange(n)))
        k = min(m, n)
        U, S, Vt = D.empty(m, k), D.empty(k), D.empty(k, n)
        work = D.empty(int(lib.ttk_svd_work(m, n)))
        lib.ttk_svd_set_timing(1)
        counters()
        t = timed(lambda: lib.ttk_svd(st, D._p(A), m, n, D._p(U), D._p(S), D._p(Vt), D._p(work)))
        c = counters()
        lib.ttk_svd_set_timing(0)
        calls = max(c[0], 1)
        print(f"{m:3d}x{n:<3d} {t:9.1f} {c[1] / calls:6.1f}  {[round(c[i] / 100.0 / calls, 1) for i in (4, 5, 6, 7)]}",
              flush=True)


if __name__ == "__main__":
    main()
