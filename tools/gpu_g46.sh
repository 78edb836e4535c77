set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTIPM_OPSTATS=1 timeout -k 10 500 python -u tools/profile_case.py maxcut maxcut_10 23 1 > gpurun_out/g46_cprof.log 2>&1 && \
cp gpurun_out/prof_maxcut_10_s23.txt gpurun_out/g46_prof_mc10_s23.txt && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g46_prof -o run -- python3 tools/run_case.py maxcut maxcut_10 23 1 > gpurun_out/g46_prof.log 2>&1 && \
mkdir -p gpurun_out/g46_prof && cp $(find /tmp/g46_prof -name "*stats.csv") gpurun_out/g46_prof/
