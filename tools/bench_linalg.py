"""Kernel-only timings (HIP events on the launch stream) of the dense factorisation kernels at
the sizes the TT-IPM path produces.  Dev tool:  python tools/bench_linalg.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402


def counters(reset=True):
    import ctypes
    buf = (ctypes.c_ulonglong * 8)()
    lib.ttk_debug_counters(buf, 1 if reset else 0)
    return list(buf)


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps  # us


def main():
    rng = np.random.default_rng(0)
    # empty kernel round trip for reference
    z = D.empty(1)
    st = D._stream()
    print(f"fill kernel (launch floor) {timed(lambda: lib.ttk_fill(st, D._p(z), 1, 0.0)):.1f}us")
    print("svd kernel-only (us) / host wrapper (us)")
    for m, n in [(2, 1), (4, 4), (8, 8), (16, 16), (32, 32), (20, 24), (64, 84), (100, 184), (156, 240), (372, 744), (868, 1024)]:
        A = D.from_numpy(rng.standard_normal((m, n)))
        k = min(m, n)
        U, S, Vt = D.empty(m, k), D.empty(k), D.empty(k, n)
        work = D.empty(int(lib.ttk_svd_work(m, n)))
        st = D._stream()
        if m > 300:
            t0 = time.perf_counter()
            D.svd(A)
            print(f"  svd {m:4d}x{n:<4d} wrapper {(time.perf_counter() - t0) * 1e6:9.1f}", flush=True)
            continue
        for kind in ("ident", "rand"):
            if kind == "ident":
                Ai = D.from_numpy(np.eye(m, n))
                counters()
                t_i = timed(lambda: lib.ttk_svd(st, D._p(Ai), m, n, D._p(U), D._p(S), D._p(Vt), D._p(work)))
                ci = counters()
        counters()
        t_k = timed(lambda: lib.ttk_svd(st, D._p(A), m, n, D._p(U), D._p(S), D._p(Vt), D._p(work)))
        c = counters()
        print(f"     identity {t_i:8.1f}us sweeps/call {ci[1] / max(ci[0], 1):.1f};  random sweeps/call "
              f"{c[1] / max(c[0], 1):.1f}  phases us (qrcp, jacobi, vectors, out): "
              f"{[round(c[k] / 100.0 / max(c[0], 1), 1) for k in (4, 5, 6, 7)]}")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            D.svd(A)
        t_h = (time.perf_counter() - t0) / 20 * 1e6
        print(f"  svd {m:4d}x{n:<4d} kernel {t_k:9.1f}  wrapper {t_h:9.1f}", flush=True)
    print("small eig phases (us per call): tridiag, multisection, inverse iteration, back-transform")
    lib.ttk_svd_set_timing(1)
    for n in [10, 40, 80, 100, 128]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        buf = D.empty(n + 1)
        st = D._stream()
        counters()
        t_x = timed(lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx)))
        c = counters()
        calls = max(c[2], 1)
        print(f"  n={n:4d} total {t_x:8.1f}  phases {[round(c[k] / 100.0 / calls, 1) for k in (4, 5, 6, 7)]}",
              flush=True)
    lib.ttk_svd_set_timing(0)
    print("eig kernel-only (us)")
    for n in [4, 10, 20, 40, 80, 100, 139, 160, 288, 500]:
        M = rng.standard_normal((n, n))
        A = D.from_numpy(M + M.T)
        ev, W = D.empty(n), D.empty(n, n)
        work = D.empty(int(lib.ttk_syev_work(n)))
        wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
        buf = D.empty(n + 1)
        st = D._stream()
        counters()
        t_x = timed(lambda: lib.ttk_syev_extreme(st, D._p(A), n, 0, D._p(buf), D._p(buf[1:]), D._p(wx)))
        c = counters()
        print(f"     multisection rounds/call {c[3] / max(c[2], 1):.1f}")
        t_j = timed(lambda: lib.ttk_syev(st, D._p(D.clone(A)), n, D._p(ev), D._p(W), D._p(work)), reps=3) \
            if n <= 300 else float("nan")
        print(f"  n={n:4d} extreme {t_x:9.1f}  jacobi {t_j:9.1f}", flush=True)


if __name__ == "__main__":
    main()
