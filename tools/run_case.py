"""Run one (problem, config, seed, rank) through the MI355X path and compare with the golden run."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from ttipm_amd.utils import run_and_record  # noqa: E402
# TTIPM_FUSED=0 -> TTK_FUSED_APPLY=0: the library reads it when each context is created (a knob set
# here, before this thread's context exists, would land on the default context only)
if os.environ.get("TTIPM_FUSED") == "0":
    os.environ["TTK_FUSED_APPLY"] = "0"

prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
key = sys.argv[5] if len(sys.argv) > 5 else f"{cfg_name}_r{rank}_s{seed}"
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", cfg_name + ".yaml")))
trace = []
t = time.time()
r = run_and_record(prob, cfg, seed, rank, trace=trace, verbose=bool(os.environ.get("TTIPM_VERBOSE")))
print("wall", time.time() - t)
g = json.load(open("tests/golden/runs.json")).get(key)
if g:
    for k in ("num_iters", "gap", "feas", "dual_feas", "ranksX", "ranksZ"):
        print(f"{k:10s} gpu={r[k]} ref={g[k]}")
    for a, b in zip(trace, g["trace"]):
        print(f"mu {a['mu']:.6e} {b['mu']:.6e}  primal {a['primal_error']:.6e} {b['primal_error']:.6e}  "
          f"sigma {a['sigma']:.4e} {b['sigma']:.4e}  ranks {a['ranksX']} {b['ranksX']}")
tag = os.environ.get("TTIPM_TAG", "")
json.dump({"result": r, "trace": trace}, open(f"gpurun_out/run_{key}{tag}.json", "w"), indent=1)
