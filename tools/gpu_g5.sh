set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTIPM_LOCAL_TRACE=1 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g5_default.log 2>&1 && \
TTIPM_LOCAL_TRACE=1 TTIPM_FUSED=0 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g5_nofused.log 2>&1 && \
timeout -k 10 120 python -u tools/check_fused.py maxcut maxcut_10 41 1 12 > gpurun_out/g5_checkfused.log 2>&1
