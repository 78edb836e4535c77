set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g51_prof -o run -- python3 tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g51_prof.log 2>&1 && \
mkdir -p gpurun_out/g51_prof && cp $(find /tmp/g51_prof -name "*stats.csv") gpurun_out/g51_prof/
