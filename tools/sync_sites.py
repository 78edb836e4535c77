"""Diagnostics (GPU): where the host waits on the device during one solve.  Every library entry
point that synchronises (names containing 'sync', ttk_read_sync, ttk_lgmres, ttk_round,
ttk_dense_schur_solve) is wrapped to record its Python call site; prints the sites by count and
the library's own ttk_sync_count per IPM iteration.

    python tools/sync_sites.py maxcut maxcut_10 41 1"""
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd import _lib  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
cfg = yaml.safe_load(open(os.path.join("configs", cfg_name + ".yaml")))
sites = collections.Counter()


class _Wrap:
    def __init__(self, name, f):
        self.name, self.f = name, f

    def __call__(self, *a):
        fr = [f for f in traceback.extract_stack()[:-1] if "ttipm" in f.filename or "interior-point" in f.filename]
        top = [f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:]]
        sites[(self.name, " < ".join(reversed(top)))] += 1
        return self.f(*a)


names = [n for n in dir(_lib.lib) if n.startswith("ttk_") and ("sync" in n or n in (
    "ttk_read_sync", "ttk_lgmres", "ttk_round", "ttk_dense_schur_solve", "ttk_lgmres_arnoldi_sync"))]
for n in names:
    setattr(_lib.lib, n, _Wrap(n, getattr(_lib.lib, n)))
run_and_record(prob, cfg, seed, rank, verbose=False)  # warm
sites.clear()
s0 = _lib.lib.ttk_sync_count()
r = run_and_record(prob, cfg, seed, rank, verbose=False)
tot = _lib.lib.ttk_sync_count() - s0
print(f"iters {r['num_iters']}  library host waits {tot} ({tot / r['num_iters']:.0f} per IPM iteration)")
for (n, site), c in sites.most_common(30):
    print(f"{c:7d} {c / r['num_iters']:8.1f}/it  {n:28s} {site}")
