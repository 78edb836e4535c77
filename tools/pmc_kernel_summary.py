"""Per-kernel sums of a rocprofv3 --pmc counter_collection.csv (SQ_* LDS counters: cycles per LDS
instruction flags misaligned or conflicting LDS traffic), printed as a small table.
    python tools/pmc_kernel_summary.py counter_collection.csv [top]"""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        k = k[:k.index("(")] if "(" in k else k
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
print(f"{'kernel':52s} {'disp':>7s} {'waveCycM':>9s} {'ldsInsM':>8s} {'ldsActM':>8s} {'act/ins':>7s} "
      f"{'conflM':>7s} {'ldsWaitM':>8s} {'valuM':>8s}")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1]["SQ_WAVE_CYCLES"])[:top]:
    ins = v["SQ_INSTS_LDS"]
    print(f"{k[:52]:52s} {len(disp[k]):7d} {v['SQ_WAVE_CYCLES'] / 1e6:9.1f} {ins / 1e6:8.2f} "
          f"{v['SQ_LDS_IDX_ACTIVE'] / 1e6:8.2f} {v['SQ_LDS_IDX_ACTIVE'] / max(ins, 1):7.1f} "
          f"{v['SQ_LDS_BANK_CONFLICT'] / 1e6:7.2f} {v['SQ_WAIT_INST_LDS'] / 1e6:8.2f} {v['SQ_INSTS_VALU'] / 1e6:8.2f}")
