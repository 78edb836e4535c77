set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g82_pytest.log 2>&1 && \
timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g82_mc10.log 2>&1 && \
timeout -k 10 300 python -u tools/run_case.py maxcut maxcut_12 80 2 > gpurun_out/g82_mc12.log 2>&1 && \
timeout -k 10 500 python -u tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g82_gm3.log 2>&1
