"""Diagnostics (GPU): phase split of the MFMA local-apply rows over the first Newton systems of a
graphm solve, on a -DTTK_MFMA_PROFILE build of the library:

    python -c "import sys; sys.path.insert(0, 'tensor-train-interior-point-method_amd'); import build; \
               build.build(out='tools/micro/libttk_mprof.so', defines=['TTK_MFMA_PROFILE'])"
    TTK_LIB_PATH=tools/micro/libttk_mprof.so python tools/mfma_phases.py graphm graphm_3 256 2 3"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd._lib import lib  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg_name, seed, rank, nmax = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
cfg = yaml.safe_load(open(os.path.join("configs", cfg_name + ".yaml")))


class _Stop(Exception):
    pass


class Trace(list):
    def append(self, item):
        super().append(item)
        if len(self) >= nmax:
            raise _Stop


out = (ctypes.c_ulonglong * 8)()
lib.ttk_mfma_profile(out, 1)
try:
    run_and_record(prob, cfg, seed, rank, trace=Trace(), verbose=False)
except _Stop:
    pass
import torch  # noqa: E402
torch.cuda.synchronize()
lib.ttk_mfma_profile(out, 0)
rows = max(out[7], 1)
names = ["staging", "stage1", "stage2", "stage3", "epilogue"]
tot = sum(out[i] for i in range(5))
if os.environ.get("TTK_VALU_PROFILE_WAIT"):  # VALU-profile build: [4] = hand-off wait inside staging, [5] = rows that waited
    names = names[:4]
    tot = sum(out[i] for i in range(4))
    print(f"hand-off waits: {out[5]} rows, {out[4] / 100.0 / max(out[5], 1):.2f} us per waiting row (inside staging)")
print(f"MFMA rows {out[7]}; per row (us): " + ", ".join(f"{n} {out[i] / 100.0 / rows:.2f}" for i, n in enumerate(names))
      + f"; total {tot / 100.0 / rows:.2f}")
