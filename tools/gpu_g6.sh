set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTIPM_OPSTATS=1 timeout -k 10 300 python -u tools/profile_case.py maxcut maxcut_10 41 1 > gpurun_out/g6_opstats.log 2>&1
