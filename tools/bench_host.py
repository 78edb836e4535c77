"""Host-side cost per call of the hot entry points (plan-cache hits), in microseconds."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402


def per_call(fn, reps=3000):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / reps * 1e6, (t2 - t0) / reps * 1e6


def main():
    P, A, Q, x = D.zeros(4, 3, 4), D.zeros(3, 4, 4, 3), D.zeros(4, 3, 4), D.zeros(4, 4, 4)
    out = D.zeros(4, 4, 4)
    a, b = D.zeros(16, 12), D.zeros(12, 16)
    c = D.zeros(16, 16)
    cases = {
        "torch.empty": lambda: torch.empty(64, dtype=torch.float64, device="cuda"),
        "D.empty": lambda: D.empty(4, 4, 4),
        "fill (ctypes)": lambda: D.fill_(c, 0.0),
        "copy_ (bind)": lambda: D.copy_(c, c),
        "matmul out= (1 GEMM)": lambda: D.matmul(a, b, out=c),
        "matmul alloc (1 GEMM)": lambda: D.matmul(a, b),
        "env fwd (3 GEMM)": lambda: D.einsum("lsr,lML,sMNS,rNR->LSR", P, x, A, x),
        "apply fused (1)": lambda: D.einsum("lsr,smnS,LSR,rnR->lmL", P, A, Q, x, out=out, fused=True),
        "apply pairwise (3)": lambda: D.einsum("lsr,smnS,LSR,rnR->lmL", P, A, Q, x, out=out),
        "dot (sync)": lambda: D.dot(c, c),
        "read (sync)": lambda: D.read(c[:1, :1]),
    }
    print(f"{'case':24s} {'host us':>9s} {'incl sync us':>13s}")
    for name, fn in cases.items():
        h, t = per_call(fn)
        print(f"{name:24s} {h:9.2f} {t:13.2f}", flush=True)
    print("launches counted", lib.ttk_launch_count())


if __name__ == "__main__":
    main()
