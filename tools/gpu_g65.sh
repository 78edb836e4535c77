set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
TTIPM_TAG=schur1 TTIPM_SCHUR_OP=1 timeout -k 10 200 python -u tools/time_solves.py maxcut maxcut_10 41 1 4 >> gpurun_out/g65.log 2>/dev/null || exit 1
TTIPM_TAG=schur0 TTIPM_SCHUR_OP=0 timeout -k 10 200 python -u tools/time_solves.py maxcut maxcut_10 41 1 4 >> gpurun_out/g65.log 2>/dev/null || exit 1
done
