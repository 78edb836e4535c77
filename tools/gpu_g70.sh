set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { timeout -k 10 300 env "$@" python -u tools/run_case.py graphm graphm_3 256 2 2>&1 | grep -E "Convergence in|Convergence after" | tr '\n' ' '; echo " <- $*"; }
run TTK_X=0 >> gpurun_out/g70.log
run TTK_FUSED_MAX_FLOPS=1e6 >> gpurun_out/g70.log
run TTK_FUSED_MAX_FLOPS=1.6e7 >> gpurun_out/g70.log
run TTK_FUSED_ENV_MAX_FLOPS=4e6 >> gpurun_out/g70.log
run TTK_FUSED_ENV_MAX_FLOPS=2.5e5 >> gpurun_out/g70.log
exit 0
