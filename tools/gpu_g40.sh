set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do for f in 0 2e5 1e6; do
TTK_FUSED_ENV_MAX_FLOPS=$f timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g40_b_${f}_$rep.json 2>/dev/null || exit 1
done; done
