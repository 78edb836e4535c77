set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_eig.py > gpurun_out/g35_eig_narrow.log 2>&1 && \
TTK_SYEV_WIDE=0 timeout -k 10 200 python -u tools/bench_eig.py > gpurun_out/g35_eig_wide.log 2>&1 && \
TTK_SYEV_WIDE=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "syev" > gpurun_out/g35_pytest.log 2>&1
