set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for f in 1e30 1e6 2e5 0; do
TTK_FUSED_ENV_MAX_FLOPS=$f timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g39_cc9_$f.log 2>&1 || exit 1
TTK_FUSED_ENV_MAX_FLOPS=$f timeout -k 10 300 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g39_mc10_$f.log 2>&1 || exit 1
done
