set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do for c in 4 8 16; do
TTIPM_TAG=chunk$c TTIPM_LGMRES_CHUNK=$c timeout -k 10 200 python -u tools/time_solves.py maxcut maxcut_10 41 1 3 2>/dev/null | grep median >> gpurun_out/g77.log || exit 1
done; done
