"""fp64 contraction GEMM throughput (ttk_einsum -> gemm_offs kernels) per shape, with torch.matmul
(rocBLAS/hipBLASLt fp64) on the same shapes as a yardstick of what the MFMA units sustain."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from tools.bench_linalg import timed  # noqa: E402

PEAK = 78.6e12


def main():
    shapes = [(1344, 1344, 1344), (2048, 2048, 2048), (4096, 4096, 4096), (172, 600, 64), (60, 40, 2580),
              (225, 688, 17), (172, 840, 64), (56, 48, 2408), (272, 196, 43), (841, 31, 15624), (336, 336, 336),
              (212, 64, 2544), (116, 64, 1160), (216, 59, 2160), (60, 44, 2700), (192, 52, 1728)]
    print(f"{'M':>5s} {'N':>5s} {'K':>6s} {'ttk_us':>9s} {'ttk_TF':>7s} {'frac':>6s} {'torch_us':>9s} {'torch_TF':>8s}")
    for M, N, K in shapes:
        a = torch.randn(M, K, dtype=torch.float64, device="cuda")
        b = torch.randn(K, N, dtype=torch.float64, device="cuda")
        c = torch.empty(M, N, dtype=torch.float64, device="cuda")
        reps = 3 if M * N * K > 1e9 else 20
        t = timed(lambda: D.matmul(a, b, out=c), reps=reps)
        err = (c - a @ b).abs().max().item() / max(1.0, (a @ b).abs().max().item())
        tt = timed(lambda: torch.matmul(a, b, out=c), reps=reps)
        fl = 2.0 * M * N * K
        print(f"{M:5d} {N:5d} {K:6d} {t:9.1f} {fl / t / 1e6:7.2f} {fl / t / 1e-6 / PEAK:6.3f} {tt:9.1f} {fl / tt / 1e6:8.2f}"
              f"  relerr {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
