"""Merge the FETCH_SIZE and WRITE_SIZE pass summaries (tools/pmc_summary.py) into the per-kernel
per-dispatch table bench.py reads (raw rocprofv3 KB per dispatch).
    python tools/pmc_merge.py fetch.json write.json out.json "<fetch cmd>" "<write cmd>" """
import json
import sys

f, w = json.load(open(sys.argv[1])), json.load(open(sys.argv[2]))
out = {"command": [sys.argv[4], sys.argv[5]],
       "note": "raw rocprofv3 FETCH_SIZE / WRITE_SIZE (KB) per dispatch, each from its own --pmc pass over "
               "the same workload; gfx950 reports FETCH_SIZE at half the bytes of wide (16 B/lane) streaming "
               "reads (MI355X_MICROARCH.md), the path's kernels issue 8 B/lane loads",
       "kernels": {}}
for k in sorted(set(f) | set(w)):
    e = {}
    if k in f and "FETCH_SIZE" in f[k]:
        e["FETCH_SIZE_KB"] = round(f[k]["FETCH_SIZE"]["mean"], 3)
        e["dispatches"] = f[k]["FETCH_SIZE"]["dispatches"]
    if k in w and "WRITE_SIZE" in w[k]:
        e["WRITE_SIZE_KB"] = round(w[k]["WRITE_SIZE"]["mean"], 3)
        e.setdefault("dispatches", w[k]["WRITE_SIZE"]["dispatches"])
    out["kernels"][k] = e
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out["kernels"].get("gemm_offs_kernel")), json.dumps(out["kernels"].get("fused_apply_kernel")))
