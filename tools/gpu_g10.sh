set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/g10_pytest.log 2>&1
timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g10_mc10.log 2>&1
export TTIPM_VERBOSE=1
timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g10_cc9.log 2>&1
timeout -k 10 400 python -u tools/run_case.py maxcut maxcut_12 80 2 > gpurun_out/g10_mc12.log 2>&1
timeout -k 10 400 python -u tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g10_gm3.log 2>&1
exit 0
