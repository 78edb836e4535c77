set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/ab_lu.log
TTK_LIB_PATH=ab/libttk_r04.so timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_old.npz > gpurun_out/ab_dump_old.log 2>&1 || { tail gpurun_out/ab_dump_old.log; exit 1; }
timeout -k 10 300 python tools/dump_kernels.py gpurun_out/ab_new.npz > gpurun_out/ab_dump_new.log 2>&1 || { tail gpurun_out/ab_dump_new.log; exit 1; }
python tools/npz_equal.py gpurun_out/ab_old.npz gpurun_out/ab_new.npz > $L 2>&1
TTK_LU_REG_PANEL=0 TTK_LU_SIZES=300,600,1000,1680,2100,3120,3600 timeout -k 10 200 python tools/bench_lu.py >> $L 2>&1 || exit 1
TTK_LU_SIZES=300,600,1000,1680,2100,3120,3600 timeout -k 10 200 python tools/bench_lu.py >> $L 2>&1 || exit 1
TTK_QR_NARROW=0 timeout -k 10 100 python tools/bench_qr_small.py >> $L 2>&1 || exit 1
timeout -k 10 100 python tools/bench_qr_small.py >> $L 2>&1 || exit 1
cat $L
