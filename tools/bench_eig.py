"""Extreme-eigenpair kernel latency per size and path (LDS small / L2 one-workgroup / multi-WG)."""
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
    print("small eig phases (us per call): tridiag, multisection, inverse iteration, back-transform")
    from tools.bench_linalg import counters
    lib.ttk_svd_set_timing(1)
    for n in [10, 40, 80, 100, 128]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        buf = D.empty(n + 1)
        counters()
        t_x = timed(lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx)))
        c = counters()
        calls = max(c[2], 1)
        print(f"  n={n:4d} total {t_x:8.1f}  phases {[round(c[k] / 100.0 / calls, 1) for k in (4, 5, 6, 7)]}",
              flush=True)
    lib.ttk_svd_set_timing(0)
    print("n      default_us   two_launch_us   lam_diff")
    for n in [4, 10, 20, 40, 80, 100, 128, 139, 160, 200, 288, 400, 504, 768, 1200]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        buf = D.empty(n + 1)
        f = lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx))  # noqa: E731
        t_d = timed(f, reps=10)
        l_d = D.read(buf[:1])[0]
        old = lib.ttk_syev_set_fused_max(0)
        t_m = timed(f, reps=5) if n > 128 else float("nan")
        l_m = D.read(buf[:1])[0]
        lib.ttk_syev_set_fused_max(old)
        print(f"{n:5d} {t_d:11.1f} {'':7s} {t_m:11.1f}  {abs(l_d - l_m):.2e}", flush=True)


if __name__ == "__main__":
    main()
