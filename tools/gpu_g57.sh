set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTK_LU_BLOCK_MIN=8 timeout -k 10 300 python -u tools/bench_lu.py > gpurun_out/g57_lu_blk.log 2>&1 && \
TTK_LU_BLOCK_MIN=100000 timeout -k 10 300 python -u tools/bench_lu.py > gpurun_out/g57_lu_old.log 2>&1 && \
TTK_LU_BLOCK_MIN=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "lu" > gpurun_out/g57_pytest.log 2>&1
