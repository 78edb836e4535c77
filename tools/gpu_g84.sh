set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/run_case.py maxcut maxcut_12 80 2 > gpurun_out/g84_mc12.log 2>&1
