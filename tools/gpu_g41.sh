set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTIPM_OPSTATS=1 timeout -k 10 500 python -u tools/profile_case.py maxcut maxcut_10 23 1 > gpurun_out/g41_cprof.log 2>&1 && \
cp gpurun_out/prof_maxcut_10_s23.txt gpurun_out/g41_prof_mc10_s23.txt
