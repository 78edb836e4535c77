set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g59_pytest.log 2>&1 && \
for rep in 1 2; do for ft in 1 0; do
TTIPM_EIG_FUSED_TAIL=$ft timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g59_mc10_${ft}_$rep.log 2>&1 || exit 1
done; done
