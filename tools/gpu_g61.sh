set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_svd_small.py > gpurun_out/g61_svd.log 2>&1
