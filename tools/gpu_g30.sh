set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g30_pytest.log 2>&1 && \
timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g30_mc10.log 2>&1 && \
TTIPM_LGMRES_CHUNK=1 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g30_mc10_chunk1.log 2>&1 && \
TTIPM_NO_BIND=1 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g30_mc10_nobind.log 2>&1 && \
timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g30_cc9.log 2>&1 && \
timeout -k 10 500 python -u tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g30_gm3.log 2>&1
