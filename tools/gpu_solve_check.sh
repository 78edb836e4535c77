#!/bin/bash
# Host-wait count and whole-solve end points on the GPU (one job):
#   gpurun -- 'bash tools/gpu_solve_check.sh TAG [SEED ...]'
# sync_sites on maxcut_10 s41, then run_case on each maxcut_10 seed (gap / feas / iterations to
# full precision, for bit-identity against the previous code).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sync_sites.py maxcut maxcut_10 41 1 > gpurun_out/${tag}_s41_sync_sites.txt 2>&1 \
  || { tail -20 gpurun_out/${tag}_s41_sync_sites.txt; exit 1; }
grep "host waits" gpurun_out/${tag}_s41_sync_sites.txt
for s in "$@"; do
  TTIPM_TAG=_$tag timeout -k 10 300 python -u tools/run_case.py maxcut maxcut_10 $s 1 > gpurun_out/${tag}_s$s.txt 2>&1 \
    || { tail -20 gpurun_out/${tag}_s$s.txt; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/run_maxcut_10_r1_s$s$(echo _$tag).json'))['result']; print($s, r['num_iters'], repr(r['gap']), repr(r['feas']))"
done
