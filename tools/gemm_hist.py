"""Record the GEMM-step shape histogram of the first N Newton systems of one run (diagnostics).
    python tools/gemm_hist.py problem config seed rank N out.txt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd._lib import lib  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg, seed, rank, nstop, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6]
config = yaml.safe_load(open(os.path.join("configs", cfg + ".yaml")))


class Stop(Exception):
    pass


class Tr(list):
    def append(self, e):
        super().append(e)
        if len(self) > nstop:
            raise Stop


import time  # noqa: E402
import torch  # noqa: E402

lib.ttk_gemm_hist(1, None)
t0 = time.time()
try:
    run_and_record(prob, config, seed, rank, trace=Tr(), verbose=False)
except Stop:
    pass
torch.cuda.synchronize()
print(f"wall to Newton system {nstop + 1}: {time.time() - t0:.2f}s", flush=True)
lib.ttk_gemm_hist(0, out.encode())
