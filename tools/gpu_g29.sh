set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/g29_bench.json 2> gpurun_out/g29_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g29_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g29_prof.log 2>&1 && \
mkdir -p gpurun_out/g29_prof && cp $(find /tmp/g29_prof -name "*stats.csv") gpurun_out/g29_prof/ && \
timeout -k 10 300 python -u tools/profile_case.py maxcut maxcut_10 41 1 > gpurun_out/g29_cprof.log 2>&1
