set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/g21_bench.json 2> gpurun_out/g21_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g21_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g21_prof.log 2>&1 && \
mkdir -p gpurun_out/g21_prof && cp $(find /tmp/g21_prof -name "*stats.csv") gpurun_out/g21_prof/ && \
TTIPM_VERBOSE=1 timeout -k 10 500 python -u tools/run_case.py graphm graphm_3 256 2 > gpurun_out/g21_gm3.log 2>&1
