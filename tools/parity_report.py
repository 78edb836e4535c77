"""Device-vs-reference parity report over the committed goldens (GPU box).

    python tools/parity_report.py [key ...]     # default: every full-solve key of runs.json

For each key: iteration counts, the first Newton-system assembly whose (mu, primal, dual,
centrality) error departs from the reference's by more than 1e-10 / 1e-6 relative, and the relative
differences of the final gap / feasibility / dual feasibility.  Prints one JSON line per key."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import yaml  # noqa: E402

RUNS = json.load(open(os.path.join(ROOT, "tests", "golden", "runs.json")))
KEYS = ("mu", "primal_error", "dual_error", "centrality_error")


def first_departure(trace, gold, tol):
    for i, (a, b) in enumerate(zip(trace, gold)):
        if a["ranksX"] != b["ranksX"]:
            return i, "ranksX"
        for k in KEYS:
            if abs(a[k] - b[k]) > tol * abs(b[k]) + 1e-300:
                return i, k
    return None


def main():
    import torch
    torch.cuda.set_device(0)
    from ttipm_amd import tt_ipm
    from ttipm_amd.utils import run_and_record
    keys = sys.argv[1:] or [k for k, v in RUNS.items() if not v.get("bounded") and "_t" not in k.split("_s")[-1]]
    for key in keys:
        g = RUNS[key]
        cfg = yaml.safe_load(open(os.path.join(ROOT, "configs", g["config"] + ".yaml")))
        old = tt_ipm.INEQ_MATVEC_BUG
        tt_ipm.INEQ_MATVEC_BUG = not g.get("fixed_ineq", True)
        trace = []
        try:
            r = run_and_record(g["problem"], cfg, g["seed"], g["rank"], trace=trace, verbose=False)
        finally:
            tt_ipm.INEQ_MATVEC_BUG = old
        out = {"key": key, "iters": [r["num_iters"], g["num_iters"]],
               "dep_1e-10": first_departure(trace, g["trace"], 1e-10),
               "dep_1e-6": first_departure(trace, g["trace"], 1e-6),
               "dep_1e-4": first_departure(trace, g["trace"], 1e-4)}
        for k in ("gap", "feas", "dual_feas"):
            out[k] = [r[k], g[k], abs(r[k] - g[k]) / abs(g[k])]
        out["per_assembly_max_rel"] = [max(abs(a[k] - b[k]) / abs(b[k]) for k in KEYS)
                                       for a, b in zip(trace, g["trace"])]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
