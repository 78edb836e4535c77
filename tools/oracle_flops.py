"""Algorithmic contraction FLOPs of one oracle solve (SURVEY.md §8(d) convention: NumPy einsum_path
greedy count per einsum call + the chained applies of every Schur operator application).  Test
tooling: prints one JSON line for comparison with bench.py's `roofline.algorithmic_flops_per_solve`.

    OPENBLAS_NUM_THREADS=1 python tools/oracle_flops.py maxcut maxcut_10 41 1"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import yaml  # noqa: E402

from oracle import problems as OP  # noqa: E402
from oracle import tt as OT  # noqa: E402

problem, cfg, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
config = yaml.safe_load(open(os.path.join(os.path.dirname(HERE), "configs", cfg + ".yaml")))
OT.ALGO = {"flops": 0.0, "calls": 0, "by_eq": {}}
res = OP.run_and_record(problem, config, seed, rank)
print(json.dumps({"problem": problem, "config": cfg, "seed": seed, "rank": rank, "num_iters": res["num_iters"],
                  "algorithmic_flops_per_solve": OT.ALGO["flops"], "calls": OT.ALGO["calls"],
                  "per_iter": OT.ALGO["flops"] / max(res["num_iters"], 1),
                  "by_eq": dict(sorted(OT.ALGO["by_eq"].items(), key=lambda kv: -kv[1][1])[:12])}))
