set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -rs --timeout 300 --timeout-method thread > gpurun_out/g64_pytest.log 2>&1 && \
for rep in 1 2; do for so in 1 0; do
TTIPM_SCHUR_OP=$so timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g64_mc10_${so}_$rep.log 2>&1 || exit 1
done; done && \
timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g64_cc9.log 2>&1
