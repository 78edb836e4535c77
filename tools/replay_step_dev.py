"""Replay one dumped step-size eigenproblem (tt_ipm TTIPM_DUMP_STEP) on the device and in the oracle
with TTIPM_EIG_DEBUG traces of every local solve.   python tools/replay_step_dev.py FILE.npz [x|z]"""
import os
import sys

os.environ["TTIPM_EIG_DEBUG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from oracle import eig as OE  # noqa: E402
from ttipm_amd import dev as D  # noqa: E402
from ttipm_amd.tt_eig import tt_max_generalised_eigen  # noqa: E402


def _tt(f, name):
    if name + "/n" not in f:
        return None
    return [f[f"{name}/{i}"].copy() for i in range(int(f[name + "/n"]))]


f = np.load(sys.argv[1])
which = sys.argv[2] if len(sys.argv) > 2 else "z"
A, Dl, x0 = (("X", "DX", "x0") if which == "x" else ("Z", "DZ", "z0"))
state = ("MT19937", f["rng_key"], int(f["rng_pos"]), int(f["rng_g"]), float(f["rng_c"]))
np.random.set_state(state)
if which == "z":  # the x call ran first and consumed draws: replay it untraced on the oracle to advance
    OE._DEBUG = False
    OE.max_generalised_eigen(_tt(f, "X"), _tt(f, "DX"), x0=_tt(f, "x0"), tol=1e-8)
    OE._DEBUG = True
st2 = np.random.get_state()
print("== oracle")
o, _ = OE.max_generalised_eigen(_tt(f, A), _tt(f, Dl), x0=_tt(f, x0), tol=1e-8)
print("oracle step", o)
np.random.set_state(st2)
up = lambda tt: None if tt is None else [D.from_numpy(c) for c in tt]  # noqa: E731
print("== device")
s, _ = tt_max_generalised_eigen(up(_tt(f, A)), up(_tt(f, Dl)), x0=up(_tt(f, x0)), tol=1e-8)
print("device step", s, "dumped", float(f["xs" if which == "x" else "zs"]))
