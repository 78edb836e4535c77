set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g7_pytest.log 2>&1
timeout -k 10 300 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g7_case.log 2>&1 && \
TTIPM_OPSTATS=1 timeout -k 10 300 python -u tools/profile_case.py maxcut maxcut_10 41 1 > gpurun_out/g7_opstats.log 2>&1
