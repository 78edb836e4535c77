set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=tensor-train-interior-point-method_amd
TTIPM_DUMP_STEP=gpurun_out/dump_default timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g3_default.log 2>&1 && \
TTIPM_DUMP_STEP=gpurun_out/dump_exnf TTK_LIB_PATH=$PWD/$L/libttk_exact.so TTIPM_FUSED=0 timeout -k 10 120 python -u tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g3_exnf.log 2>&1 && \
timeout -k 10 300 python -u tools/profile_case.py maxcut maxcut_10 41 1 > gpurun_out/g3_cprof.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g3_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g3_prof.log 2>&1 && \
mkdir -p gpurun_out/g3_prof && cp $(find /tmp/g3_prof -name "*stats.csv") gpurun_out/g3_prof/
