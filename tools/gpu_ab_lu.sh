#!/bin/bash
# A/B of the LU / QR kernel changes on the GPU box (one job): kernel outputs bit for bit against the
# round-4 library (tools/dump_kernels.py + npz_equal.py), then tools/bench_lu.py with the new paths off
# (env $OFF, e.g. TTK_LU_SWAP_U12=0) and on.   gpurun -- 'bash tools/gpu_ab_lu.sh TTK_LU_SWAP_U12=0'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/ab_lu.log
OFF=${1:-TTK_LU_REG_PANEL=0}
TTK_LIB_PATH=ab/libttk_r04.so timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_old.npz > gpurun_out/ab_dump_old.log 2>&1 || { tail gpurun_out/ab_dump_old.log; exit 1; }
timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_new.npz > gpurun_out/ab_dump_new.log 2>&1 || { tail gpurun_out/ab_dump_new.log; exit 1; }
python tools/npz_equal.py gpurun_out/ab_old.npz gpurun_out/ab_new.npz > $L 2>&1
echo "== $OFF" >> $L
env $OFF TTK_LU_SIZES=300,600,1000,1680,2100,3120,3600 timeout -k 10 200 python tools/bench_lu.py >> $L 2>&1 || exit 1
echo "== default" >> $L
TTK_LU_SIZES=300,600,1000,1680,2100,3120,3600 timeout -k 10 200 python tools/bench_lu.py >> $L 2>&1 || exit 1
cat $L
