"""Dump the outputs of a fixed set of kernel calls (extreme eigenpairs, offset-table GEMMs) on seeded
inputs, so two library builds can be compared bit for bit:

    TTK_LIB_PATH=old.so python tools/dump_kernels.py gpurun_out/a.npz
    python tools/dump_kernels.py gpurun_out/b.npz        # then compare the two files on the host"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd._lib import lib  # noqa: E402


def main(path):
    rng = np.random.default_rng(0)
    st = D._stream()
    out = {}
    for n in [3, 5, 10, 17, 40, 63, 64, 80, 100, 127, 128, 139, 200]:
        for which in (0, 1):
            M = rng.standard_normal((n, n))
            A = D.from_numpy(M + M.T)
            wx = D.empty(int(lib.ttk_syev_extreme_work(n)))
            buf = D.empty(n + 1)
            D.check(lib.ttk_syev_extreme(st, D._p(A), n, which, D._p(buf), D._p(buf[1:]), D._p(wx)), "syev")
            out[f"syev_{n}_{which}"] = D.read(buf)
    for M_, N_, K_ in [(212, 64, 2544), (60, 44, 2700), (30, 20, 7), (172, 600, 64), (336, 336, 336), (700, 650, 520)]:
        a = torch.randn(M_, K_, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(K_))
        b = torch.randn(K_, N_, dtype=torch.float64, device="cuda", generator=torch.Generator("cuda").manual_seed(N_))
        out[f"mm_{M_}_{N_}_{K_}"] = D.read(D.matmul(a, b))
        out[f"mmT_{M_}_{N_}_{K_}"] = D.read(D.matmul(b.t(), a.t()))
    torch.cuda.synchronize()
    np.savez(path, **out)
    print("dumped", len(out), "arrays to", path)


if __name__ == "__main__":
    main(sys.argv[1])
