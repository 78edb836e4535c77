set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/bench_host.py > gpurun_out/g36_host.log 2>&1 && \
timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g36_mc10.log 2>&1
