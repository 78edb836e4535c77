set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/g52_gemm.log 2>&1
