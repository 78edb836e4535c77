set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for mk in 256 128 64; do
TTK_SPLITK_MINK=$mk timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/g68_gemm_$mk.log 2>&1 || exit 1
done
