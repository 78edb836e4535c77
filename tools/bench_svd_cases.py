"""Time the device SVD on dumped real unfoldings (.svd_cases/*.npy; dev tool)."""
import glob
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402
import ctypes  # noqa: E402

lib.ttk_svd_set_timing(1)

for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else ".svd_cases/*.npy")):
    A = np.load(f)
    dA = D.from_numpy(A)
    D.svd(dA)
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 8)()
    lib.ttk_debug_counters(buf, 1)
    t = time.perf_counter()
    U, S, Vt, s = D.svd(dA)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    ref = np.linalg.svd(A, compute_uv=False)
    U, Vt = D.read(U), D.read(Vt)
    err = np.abs((U * s) @ Vt - A).max() / np.abs(A).max()
    print(f"{f} {A.shape} {dt * 1e3:8.1f} ms  sv err {np.max(np.abs(s - ref)) / ref[0]:.2e}  recon {err:.2e}  "
          f"orthU {np.abs(U.T @ U - np.eye(U.shape[1])).max():.2e}", flush=True)
    lib.ttk_debug_counters(buf, 1)
    if buf[0]:
        print(f"     phases us (qrcp, jacobi, post-jacobi, vectors): {[round(buf[k] / 100.0, 1) for k in (4, 5, 6, 7)]} "
              f"sweeps {buf[1]}  shader clock {buf[2] / max(buf[3], 1) * 0.1:.2f} GHz", flush=True)
