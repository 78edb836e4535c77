"""Device-vs-reference parity report over the committed goldens (GPU box).

    python tools/parity_report.py [key ...]     # default: every full-solve key of runs.json

For each key: iteration counts, per Newton-system assembly the device's max relative difference
from the 1-thread reference over (mu, primal, dual, centrality) beside the reference's own
1-vs-8-thread spread (when the `_t8` twin exists), the first assembly that leaves
max(FLOOR, 50 x spread), and the relative differences of the final gap / feasibilities.
Prints one JSON line per key (the per-assembly report committed under profiles/)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import yaml  # noqa: E402

RUNS = json.load(open(os.path.join(ROOT, "tests", "golden", "runs.json")))
KEYS = ("mu", "primal_error", "dual_error", "centrality_error")
FLOOR = 1e-9  # relative: the device's first assemblies differ at ~1e-13 (GEMM association)


def rel(a, b):
    return max(abs(a[k] - b[k]) / abs(b[k]) for k in KEYS)


def first_departure(trace, gold, tol):
    for i, (a, b) in enumerate(zip(trace, gold)):
        if a["ranksX"] != b["ranksX"]:
            return i, "ranksX"
        for k in KEYS:
            if abs(a[k] - b[k]) > tol * abs(b[k]) + 1e-300:
                return i, k
    return None


def spread_report(trace, key):
    g = RUNS[key]["trace"]
    tw = RUNS.get(key + "_t8")
    dev = [rel(a, b) for a, b in zip(trace, g)]
    out = {"per_assembly_dev_vs_t1": dev}
    if tw:
        sp = [rel(b, c) for b, c in zip(g, tw["trace"])]
        out["per_assembly_ref_spread"] = sp
        first_out = None
        for i, (dv, s) in enumerate(zip(dev, sp)):
            if s > 1e-3:
                break
            if dv > max(FLOOR, 50 * s):
                first_out = i
                break
        out["first_outside_50x_spread"] = first_out
        out["checked_assemblies"] = next((i for i, s in enumerate(sp) if s > 1e-3), len(sp))
    return out


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
            if key + "_t8" in RUNS:
                out[k + "_t8"] = RUNS[key + "_t8"][k]
        out.update(spread_report(trace, key))
        out["trace"] = [{k: a[k] for k in KEYS + ("sigma", "ranksX")} for a in trace]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
