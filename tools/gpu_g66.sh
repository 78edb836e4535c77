set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/profile_case.py maxcut maxcut_10 41 1 > gpurun_out/g66_cprof.log 2>&1 && \
cp gpurun_out/prof_maxcut_10_s41.txt gpurun_out/g66_prof_mc10.txt
