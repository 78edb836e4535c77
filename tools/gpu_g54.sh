set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TTK_GEMM64_KS=32 timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/g54_gemm32.log 2>&1 && \
TTK_GEMM64_KS=16 timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/g54_gemm16.log 2>&1
