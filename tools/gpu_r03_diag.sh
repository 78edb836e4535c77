#!/bin/bash
# round-3 diagnostics on the GPU box: local-solve traces, kernel stats of single solves, parity report
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
R=$PWD
mkdir -p gpurun_out
for s in 41 14; do
  TTIPM_LOCAL_TRACE=1 timeout -k 10 300 python tools/time_solves.py maxcut maxcut_10 $s 1 1 > gpurun_out/lt_s$s.log 2>&1 || exit 1
done
for s in 41 14; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ps$s -o run -- \
     python3 $R/tools/time_solves.py maxcut maxcut_10 $s 1 1 > $R/gpurun_out/ps$s.log 2>&1) || exit 1
  for f in $(find /tmp/ps$s -name "*kernel_stats.csv"); do cp $f gpurun_out/ps${s}_kernel_stats.csv; done
done
timeout -k 10 900 python -u tools/parity_report.py > gpurun_out/r03_parity_report.jsonl 2> gpurun_out/r03_parity_report.err || exit 1
echo done
