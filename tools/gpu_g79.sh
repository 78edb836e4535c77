set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g79_pytest.log 2>&1 && \
for rep in 1 2; do
TTIPM_TAG=join timeout -k 10 200 python -u tools/time_solves.py maxcut maxcut_10 41 1 3 2>/dev/null | grep median >> gpurun_out/g79.log || exit 1
done
