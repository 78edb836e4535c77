set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "syev" > gpurun_out/g13_pytest.log 2>&1 && \
timeout -k 10 240 python -u tools/bench_linalg.py > gpurun_out/g13_linalg.log 2>&1 && \
timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g13_mc10.log 2>&1
