"""Run the CPU oracle on one (problem, config, seed, rank) and print each Newton-system trace entry
as it happens (diagnostics for configs without a committed golden run).
    python tools/oracle_trace.py maxcut maxcut_12 80 2"""
import json
import os
import sys
import time

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import yaml  # noqa: E402

from oracle.problems import run_and_record  # noqa: E402


class Printing(list):
    def append(self, e):
        super().append(e)
        print(time.strftime("%H:%M:%S"), json.dumps({k: e[k] for k in e if not k.startswith("ranks")}),
              "ranksX", e.get("ranksX"), flush=True)


prob, cfg_name, seed, rank = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
cfg = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs",
                                       cfg_name + ".yaml")))
r = run_and_record(prob, cfg, seed, rank, trace=Printing())
print(json.dumps(r), flush=True)
