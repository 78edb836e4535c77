"""Re-evaluate a saved tools/parity_report.py output (JSON lines) against the CURRENT goldens and
twins (tests/golden/runs.json) with the whole-solve parity policy of tests/parity_policy.py -- e.g.
after more reference twins were generated.  python tools/parity_offline.py REPORT.jsonl"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests import parity_policy as P  # noqa: E402

for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    rep = json.loads(line)
    key = rep["key"]
    r = rep.get("result") or {"num_iters": rep["iters"][0], "gap": rep["gap"][0], "feas": rep["feas"][0],
                               "dual_feas": rep["dual_feas"][0], "ranksX": None, "ranksZ": None}
    cum, checked, stable = P.reference_noise(key)
    try:
        name, per, _ = P.check_against_reference_runs(key, rep["trace"], r)
        verdict = f"pass: follows {name}"
    except AssertionError as e:
        verdict = f"FAIL: {str(e)[:160]}"
    ntw = sum(1 for x in P.ALL_TWINS if key + x in P.RUNS)
    print(f"{key:34s} iters dev {r['num_iters']:3d} gap {r['gap']:.4e}  twins {ntw:2d}  checked {checked:2d}  "
          f"{'stable' if stable else 'branching'}  {verdict}")
