"""Record (op, output ranks, output norm) for every TT-algebra call until the first N Newton-system
assemblies of one run -- diff a GPU run against the CPU-emulated host path to find the first op
whose result differs.   python tools/trace_ops.py [--emu] problem config seed rank N out.json"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
args = [a for a in sys.argv[1:] if a not in ("--emu", "--create")]
if "--emu" in sys.argv:
    from tests.emu_ttk import emulated_ttipm
    emulated_ttipm()
import numpy as np  # noqa: E402
import yaml  # noqa: E402

from ttipm_amd import tt_ops as T  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg, seed, rank, nstop, out = args[0], args[1], int(args[2]), int(args[3]), int(args[4]), args[5]
config = yaml.safe_load(open(os.path.join("configs", cfg + ".yaml")))
LOG = []
ACTIVE = ["--create" in sys.argv]  # --create: also log the problem generator's ops


def wrap(name):
    f = getattr(T, name)

    def g(*a, **k):
        r = f(*a, **k)
        if ACTIVE[0] and isinstance(r, list) and r and hasattr(r[0], "shape"):
            ACTIVE[0] = False
            try:
                nrm = float(np.sqrt(max(T.tt_inner_prod(r, r), 0.0)))
            finally:
                ACTIVE[0] = True
            LOG.append([name, [int(c.shape[-1]) for c in r[:-1]], nrm])
        return r
    setattr(T, name, g)


for n in ("tt_rank_reduce", "tt_psd_rank_reduce", "tt_fast_matrix_vec_mul", "tt_fast_mat_mat_mul", "tt_add",
          "tt_sub", "tt_scale", "tt_fast_hadamard", "tt_rl_orthogonalise"):
    wrap(n)


class Stop(Exception):
    pass


class Tr(list):
    def append(self, e):
        super().append(e)
        LOG.append(["TRACE", {k: e[k] for k in ("mu", "primal_error", "dual_error", "centrality_error")}])
        if len(self) >= nstop:
            raise Stop


from ttipm_amd import utils as U  # noqa: E402

_orig_solve = U.solve


def solve(*a, **k):
    ACTIVE[0] = True
    return _orig_solve(*a, **k)


U.solve = solve
try:
    run_and_record(prob, config, seed, rank, trace=Tr(), verbose=False)
except Stop:
    pass
json.dump(LOG, open(out, "w"))
print("ops logged", len(LOG))
