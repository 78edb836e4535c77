set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/profile_case.py maxcut maxcut_10 41 1 > gpurun_out/g12_cprof.log 2>&1
