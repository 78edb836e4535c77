set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/gemm_hist.py graphm graphm_3 256 2 2 gpurun_out/gemm_hist_gm3.txt > gpurun_out/g24_hist.log 2>&1
timeout -k 10 240 python -u tools/bench_linalg.py > gpurun_out/g24_linalg.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 300 --timeout-method thread -k "syev" > gpurun_out/g24_pytest.log 2>&1
exit 0
