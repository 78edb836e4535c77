set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTIPM_EIG_DEBUG=1 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g17_mc10.log 2>&1
TTIPM_EIG_DEBUG=1 timeout -k 10 200 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g17_cc9.log 2>&1
TTIPM_OPSTATS=1 timeout -k 10 300 python -u tools/profile_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g17_cprof.log 2>&1
exit 0
