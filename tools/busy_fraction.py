"""GPU busy fraction of a profiled run: the union of kernel execution intervals over the wall span of
the kernel trace (rocprofv3 --kernel-trace CSV), and the idle gaps' distribution -- how much of a
solve's wall the device spends waiting for the host.
    python tools/busy_fraction.py DIR_WITH_kernel_trace.csv [t_from_s]"""
import csv
import glob
import os
import sys

import numpy as np

path = sys.argv[1]
f = path if path.endswith(".csv") else glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
st, en = [], []
with open(f) as fh:
    for r in csv.DictReader(fh):
        st.append(int(r["Start_Timestamp"]))
        en.append(int(r["End_Timestamp"]))
st, en = np.array(st), np.array(en)
o = np.argsort(st)
st, en = st[o], en[o]
if len(sys.argv) > 2:  # skip warm-up: keep kernels from t_from seconds after the first one
    keep = st >= st[0] + float(sys.argv[2]) * 1e9
    st, en = st[keep], en[keep]
busy, cur_s, cur_e, gaps = 0, st[0], en[0], []
for s, e in zip(st[1:], en[1:]):
    if s > cur_e:
        busy += cur_e - cur_s
        gaps.append(s - cur_e)
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = en.max() - st[0]
g = np.array(gaps) / 1e3
print(f"kernels {len(st)}  span {span / 1e9:.3f} s  busy {busy / 1e9:.3f} s ({100 * busy / span:.1f} %)  "
      f"sum of durations {(en - st).sum() / 1e9:.3f} s")
print(f"idle gaps {len(g)}: total {g.sum() / 1e6:.3f} s, median {np.median(g):.1f} us, p90 {np.percentile(g, 90):.1f} us, "
      f">50us: {int((g > 50).sum())} ({g[g > 50].sum() / 1e6:.3f} s), >200us: {int((g > 200).sum())} ({g[g > 200].sum() / 1e6:.3f} s)")
