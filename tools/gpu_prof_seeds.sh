#!/bin/bash
# rocprofv3 --kernel-trace --stats of one maxcut_10 solve per seed (tools/run_case.py), summaries to gpurun_out/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
for s in 23 14 35; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05c_s$s -o run -- python3 tools/run_case.py maxcut maxcut_10 $s 1 > gpurun_out/r05c_s${s}_rocprof.log 2>&1 || exit 1
  for f in $(find /tmp/r05c_s$s -name "*kernel_stats.csv"); do cp $f gpurun_out/r05c_s${s}_kernel_stats.csv; done
done
