"""Shape histogram of the dense factorisations in whole solves (ttk_linalg_hist; diagnostics: every
recorded call is bracketed by two stream synchronisations, so the solve itself runs slower).
    python tools/linalg_hist.py problem config rank out.txt seed [seed ...]
prints the entries sorted by total time."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd._lib import lib  # noqa: E402
from ttipm_amd.utils import run_and_record  # noqa: E402

prob, cfg, rank, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
seeds = [int(s) for s in sys.argv[5:]]
config = yaml.safe_load(open(os.path.join("configs", cfg + ".yaml")))
lib.ttk_linalg_hist(1, None)
iters = 0
for s in seeds:
    r = run_and_record(prob, config, s, rank, verbose=False)
    iters += r["num_iters"]
    print(f"seed {s}: {r['num_iters']} iterations, gap {r['gap']:.6e}", flush=True)
lib.ttk_linalg_hist(0, out.encode())
rows = [ln.split() for ln in open(out).read().splitlines()[1:]]
rows.sort(key=lambda r: -float(r[5]))
tot = sum(float(r[5]) for r in rows)
print(f"{iters} IPM iterations; recorded {tot / 1e6:.2f} s (synchronised)")
print(f"{'kind':13s} {'a':>5s} {'b':>5s} {'path':>5s} {'calls':>7s} {'calls/it':>8s} {'us/call':>9s} {'share':>6s}")
for k, a, b, p, c, us in rows[:60]:
    print(f"{k:13s} {a:>5s} {b:>5s} {p:>5s} {c:>7s} {int(c) / iters:8.1f} {float(us) / int(c):9.1f} {float(us) / tot:6.1%}")
