set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/g8_pytest.log 2>&1
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/g8_bench.json 2> gpurun_out/g8_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/g8_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g8_prof.log 2>&1 && \
mkdir -p gpurun_out/g8_prof && cp $(find /tmp/g8_prof -name "*stats.csv") gpurun_out/g8_prof/
