set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d /tmp/pmc_fetch -o run -- python3 tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g20_fetch.log 2>&1 && \
python3 tools/pmc_summary.py /tmp/pmc_fetch gpurun_out/pmc_fetch_summary.json > gpurun_out/g20_fetch_sum.log 2>&1 && \
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d /tmp/pmc_write -o run -- python3 tools/run_case.py maxcut maxcut_10 41 1 > gpurun_out/g20_write.log 2>&1 && \
python3 tools/pmc_summary.py /tmp/pmc_write gpurun_out/pmc_write_summary.json > gpurun_out/g20_write_sum.log 2>&1
