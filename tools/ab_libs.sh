#!/bin/bash
# A/B of two libttk builds on the GPU box (one job): kernel outputs bit for bit (tools/dump_kernels.py),
# then repeated solves of the given maxcut_10 seeds with each library (tools/time_solves.py: median
# s/IPM-iter and the final gap, which must agree to the last digit).
#   gpurun -- 'bash tools/ab_libs.sh ab/libttk_old.so "35 41"'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
old=$1; seeds=${2:-"35 41"}; reps=${3:-3}
mkdir -p gpurun_out
TTK_LIB_PATH=$old timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_old.npz > gpurun_out/ab_dump_old.log 2>&1 || { tail gpurun_out/ab_dump_old.log; exit 1; }
timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_new.npz > gpurun_out/ab_dump_new.log 2>&1 || { tail gpurun_out/ab_dump_new.log; exit 1; }
python tools/npz_equal.py gpurun_out/ab_old.npz gpurun_out/ab_new.npz
for s in $seeds; do
  TTIPM_TAG="old s$s" TTK_LIB_PATH=$old timeout -k 10 300 python tools/time_solves.py maxcut maxcut_10 $s 1 $reps 2>&1 | grep median || exit 1
  TTIPM_TAG="new s$s" timeout -k 10 300 python tools/time_solves.py maxcut maxcut_10 $s 1 $reps 2>&1 | grep median || exit 1
done
