set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=tensor-train-interior-point-method_amd
timeout -k 10 120 python -u tools/replay_step_dev.py diag/exnf_009.npz z > gpurun_out/g4_fast.log 2>&1 && \
TTK_LIB_PATH=$PWD/$L/libttk_exact.so timeout -k 10 120 python -u tools/replay_step_dev.py diag/exnf_009.npz z > gpurun_out/g4_exact.log 2>&1
