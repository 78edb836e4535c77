set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g18_prof -o run -- python3 tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g18_prof.log 2>&1 && \
mkdir -p gpurun_out/g18_prof && cp $(find /tmp/g18_prof -name "*stats.csv") gpurun_out/g18_prof/
