set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for f in 1e30 4e6 1e6; do
TTK_FUSED_MAX_FLOPS=$f timeout -k 10 100 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g27_mc10_$f.log 2>&1
TTK_FUSED_MAX_FLOPS=$f timeout -k 10 200 python -u tools/gemm_hist.py graphm graphm_3 256 2 3 /tmp/h.txt > gpurun_out/g27_gm3_$f.log 2>&1
done
exit 0
