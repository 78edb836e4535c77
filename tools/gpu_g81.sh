set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { timeout -k 10 300 env "$@" python -u tools/run_case.py maxcut maxcut_12 80 2 2>&1 | grep -E "Convergence in|Convergence after" | tr '\n' ' '; echo " <- $*"; }
run TTK_X=0 >> gpurun_out/g81.log
run TTK_SPLITK_MINK=256 >> gpurun_out/g81.log
run TTK_LU_BLOCK_MIN=100000 >> gpurun_out/g81.log
run TTK_SPLITK_MINK=256 TTK_LU_BLOCK_MIN=100000 >> gpurun_out/g81.log
run TTIPM_FUSED_ENV=0 >> gpurun_out/g81.log
exit 0
