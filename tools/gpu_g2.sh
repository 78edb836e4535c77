set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=tensor-train-interior-point-method_amd
timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g2_default.log 2>&1 && \
TTIPM_FUSED=0 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g2_nofused.log 2>&1 && \
TTK_LIB_PATH=$PWD/$L/libttk_exact.so timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g2_exact.log 2>&1 && \
TTK_LIB_PATH=$PWD/$L/libttk_exact.so TTIPM_FUSED=0 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g2_exact_nofused.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/g2_bench.json 2> gpurun_out/g2_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g2_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g2_prof.log 2>&1 && mkdir -p gpurun_out/g2_prof && find /tmp/g2_prof -name "*stats.csv" -exec cp {} gpurun_out/g2_prof/ ;
