set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "lu" > gpurun_out/g58_pytest.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_lu.py > gpurun_out/g58_lu.log 2>&1
