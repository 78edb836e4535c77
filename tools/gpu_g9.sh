set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export TTIPM_VERBOSE=1
timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g9_cc9.log 2>&1
timeout -k 10 400 python -u tools/run_case.py maxcut maxcut_12 80 2 > gpurun_out/g9_mc12.log 2>&1
timeout -k 10 400 python -u tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g9_gm3.log 2>&1
exit 0
