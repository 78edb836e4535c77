"""Extreme-eigenpair kernel latency per size and path (LDS small / L2 one-workgroup / multi-WG)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402
from tools.bench_linalg import timed  # noqa: E402


def step_phases():
    """syev_small_kernel's tridiagonalisation, wave 0's cycles per Householder step by phase (timing 2)."""
    from tools.bench_linalg import counters
    rng = np.random.default_rng(0)
    st = D._stream()
    lib.ttk_svd_set_timing(2)
    print("cycles per step (wave 0): symv, barrier1, K, rank-2 rows, reflector, barrier2")
    for n in [10, 40, 63, 64, 80, 100, 128]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        buf = D.empty(n + 1)
        f = lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx))  # noqa: E731
        f()
        torch.cuda.synchronize()
        counters()
        reps = 20
        t = timed(f, reps=reps)
        c = counters()
        steps = (reps + 1) * (n - 2)
        print(f"  n={n:4d} total {t:8.1f} us  " + " ".join(f"{c[k] / steps:7.0f}" for k in range(6)), flush=True)
    lib.ttk_svd_set_timing(0)


def totals():
    """Default-path latency per n (no timers), for A/B across TTK_SYEV_VAR settings."""
    rng = np.random.default_rng(0)
    st = D._stream()
    out = []
    for n in [10, 20, 40, 63, 64, 80, 100, 128]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        buf = D.empty(n + 1)
        out.append(timed(lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx)),
                         reps=20))
    print("totals_us " + " ".join(f"{t:7.1f}" for t in out), flush=True)


def tri_one():
    """One-workgroup tridiagonalisation (TTK_KNOB_TRI_ONE) against one launch per Householder step:
    latency per n and the eigenpair bits (must be identical)."""
    from ttipm_amd import _lib
    rng = np.random.default_rng(0)
    st = D._stream()
    print("n      one_wg_us  per_step_us  identical")
    for n in [129, 144, 160, 192, 224, 256, 257, 288, 320, 384, 448, 512]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        res, ts = [], []
        for v in (512, 0):
            lib.ttk_ctx_set_knob(None, _lib.KNOB_TRI_ONE, v, None)
            buf = D.empty(n + 1)
            ts.append(timed(lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx)),
                            reps=20))
            res.append(D.read(buf))
        lib.ttk_ctx_set_knob(None, _lib.KNOB_TRI_ONE, 512, None)
        print(f"{n:5d} {ts[0]:10.1f} {ts[1]:12.1f}  {bool(np.array_equal(res[0], res[1]))}", flush=True)


def main():
    if "--tri" in sys.argv:
        return tri_one()
    if "--steps" in sys.argv:
        return step_phases()
    if "--totals" in sys.argv:
        return totals()
    rng = np.random.default_rng(0)
    st = D._stream()
    print("small eig phases (us per call): tridiag, multisection, inverse iteration, back-transform")
    from tools.bench_linalg import counters
    lib.ttk_svd_set_timing(1)
    for n in [10, 40, 63, 64, 80, 100, 128]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        buf = D.empty(n + 1)
        counters()
        t_x = timed(lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx)))
        c = counters()
        calls = max(c[2], 1)
        print(f"  n={n:4d} total {t_x:8.1f}  phases {[round(c[k] / 100.0 / calls, 1) for k in (4, 5, 6, 7)]}"
              f"  multisection rounds {c[3] / calls:.1f}", flush=True)
    lib.ttk_svd_set_timing(0)
    if "--phases" in sys.argv:
        return
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
