set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/g1_pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/g1_bench.json 2> gpurun_out/g1_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/g1_prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g1_prof.log 2>&1
