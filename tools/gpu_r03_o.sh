set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_abi.py -x -q -k "lu or dense or rcond" --timeout 300 --timeout-method thread > gpurun_out/o_tests.log 2>&1 || { tail -30 gpurun_out/o_tests.log; exit 1; }
tail -2 gpurun_out/o_tests.log
TTK_LU_SIZES=200,700,1400,2200 timeout -k 10 300 python tools/bench_lu.py > gpurun_out/o_bench_lu.txt 2>&1 || { tail gpurun_out/o_bench_lu.txt; exit 1; }
cat gpurun_out/o_bench_lu.txt
for s in 23 14 41; do
  timeout -k 10 300 python tools/time_solves.py maxcut maxcut_10 $s 1 2 > gpurun_out/o_ts_$s.log 2>&1 || { tail gpurun_out/o_ts_$s.log; exit 1; }
  grep -E "median" gpurun_out/o_ts_$s.log
done
