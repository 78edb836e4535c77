set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g75_pytest.log 2>&1 && \
for rep in 1 2; do
TTIPM_TAG=chunk timeout -k 10 200 python -u tools/time_solves.py maxcut maxcut_10 41 1 4 2>/dev/null | grep median >> gpurun_out/g75.log || exit 1
done && \
timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g75_cc9.log 2>&1
