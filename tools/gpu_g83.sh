set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/g83_bench.json 2> gpurun_out/g83_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g83_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g83_prof.log 2>&1 && \
mkdir -p gpurun_out/g83_prof && cp $(find /tmp/g83_prof -name "*stats.csv") gpurun_out/g83_prof/ && \
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc_fetch -o run -- python3 tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g83_fetch.log 2>&1 && \
python3 tools/pmc_summary.py /tmp/pmc_fetch gpurun_out/g83_pmc_fetch.json > gpurun_out/g83_fetch_sum.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pmc_write -o run -- python3 tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g83_write.log 2>&1 && \
python3 tools/pmc_summary.py /tmp/pmc_write gpurun_out/g83_pmc_write.json > gpurun_out/g83_write_sum.log 2>&1
