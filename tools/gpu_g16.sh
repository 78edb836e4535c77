set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/g16_pytest.log 2>&1
timeout -k 10 600 python -u bench.py --steps 1 --warmup 1 > gpurun_out/g16_bench.json 2> gpurun_out/g16_bench.err
export TTIPM_VERBOSE=1
timeout -k 10 400 python -u tools/run_case.py maxcut maxcut_12 80 2 > gpurun_out/g16_mc12.log 2>&1
timeout -k 10 300 python -u tools/run_case.py corr_clust corr_clust_9 764 1 > gpurun_out/g16_cc9.log 2>&1
exit 0
