#!/bin/bash
# A/B of syev_small_kernel variants on the GPU box (one job): kernel outputs bit for bit against the
# round-4 library (dump_kernels.py + npz_equal.py, TTK_SYEV_VAR default), then the per-step phase
# split (bench_eig.py --steps) per TTK_SYEV_VAR value.   gpurun -- 'bash tools/gpu_ab_eig.sh 0 1 2 4 7'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/ab_eig.log
TTK_LIB_PATH=ab/libttk_r04.so timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_old.npz > gpurun_out/ab_dump_old.log 2>&1 || { tail gpurun_out/ab_dump_old.log; exit 1; }
timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_new.npz > gpurun_out/ab_dump_new.log 2>&1 || { tail gpurun_out/ab_dump_new.log; exit 1; }
python tools/npz_equal.py gpurun_out/ab_old.npz gpurun_out/ab_new.npz > $L 2>&1
for v in "$@"; do
  echo "== TTK_SYEV_VAR=$v" >> $L
  TTK_SYEV_VAR=$v timeout -k 10 200 python tools/bench_eig.py --steps >> $L 2>&1 || exit 1
  TTK_SYEV_VAR=$v timeout -k 10 200 python tools/bench_eig.py --totals >> $L 2>&1 || exit 1
done
cat $L
