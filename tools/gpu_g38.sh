set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTIPM_FUSED_ENV=0 timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g38_cc9_pair.log 2>&1 && \
timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g38_cc9.log 2>&1 && \
timeout -k 10 500 python -u tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g38_gm3.log 2>&1 && \
TTIPM_FUSED_ENV=0 timeout -k 10 500 python -u tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g38_gm3_pair.log 2>&1
