set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_lu.py > gpurun_out/g43_lu_blk.log 2>&1 && \
TTK_LU_BLOCK_MIN=100000 timeout -k 10 300 python -u tools/bench_lu.py > gpurun_out/g43_lu_old.log 2>&1 && \
for rep in 1 2; do for m in 96 100000; do
TTK_LU_BLOCK_MIN=$m timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g43_mc10_${m}_$rep.log 2>&1 || exit 1
done; done
