set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g60_pytest.log 2>&1 && \
for rep in 1 2 3; do
timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g60_mc10_$rep.log 2>&1 || exit 1
done
