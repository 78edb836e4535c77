"""Replay dumped step-size eigenproblems (tt_ipm TTIPM_DUMP_STEP) through the oracle on the CPU.

    python tools/replay_step.py DUMP_DIR
For each call: the device step sizes (xs, zs) next to the oracle's `max_generalised_eigen` on the
same X/DX/Z/DZ, warm starts and MT19937 state."""
import glob
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import eig as OE  # noqa: E402


def _tt(f, name):
    if name + "/n" not in f:
        return None
    return [f[f"{name}/{i}"].copy() for i in range(int(f[name + "/n"]))]


for path in sorted(glob.glob(os.path.join(sys.argv[1], "step_*.npz"))):
    f = np.load(path)
    np.random.set_state(("MT19937", f["rng_key"], int(f["rng_pos"]), int(f["rng_g"]), float(f["rng_c"])))
    ox, _ = OE.max_generalised_eigen(_tt(f, "X"), _tt(f, "DX"), x0=_tt(f, "x0"), tol=1e-8)
    oz, _ = OE.max_generalised_eigen(_tt(f, "Z"), _tt(f, "DZ"), x0=_tt(f, "z0"), tol=1e-8)
    xs, zs = float(f["xs"]), float(f["zs"])
    print(f"{os.path.basename(path)}  xs dev {xs:.10e} oracle {ox:.10e} rel {abs(xs - ox) / max(abs(ox), 1e-300):.2e}"
          f"   zs dev {zs:.10e} oracle {oz:.10e} rel {abs(zs - oz) / max(abs(oz), 1e-300):.2e}")
