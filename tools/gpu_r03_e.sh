set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q -k "lanczos or test_syev_extreme or dense_schur or schur or lgmres" --timeout 120 --timeout-method thread > gpurun_out/e_tests.log 2>&1 || { tail -30 gpurun_out/e_tests.log; exit 1; }
tail -2 gpurun_out/e_tests.log
timeout -k 10 300 python tools/bench_lanczos.py > gpurun_out/e_bench_lanczos.log 2>&1 || { tail gpurun_out/e_bench_lanczos.log; exit 1; }
cat gpurun_out/e_bench_lanczos.log
for s in 41 14 35; do
  echo "== s$s dense_op=1"; timeout -k 10 300 python tools/time_solves.py maxcut maxcut_10 $s 1 2 > gpurun_out/e_ts_$s.log 2>&1 || { tail gpurun_out/e_ts_$s.log; exit 1; }
  grep -E "median|lanczos|iters" gpurun_out/e_ts_$s.log
  echo "== s$s dense_op=0"; TTIPM_DENSE_OP=0 timeout -k 10 300 python tools/time_solves.py maxcut maxcut_10 $s 1 2 > gpurun_out/e_ts0_$s.log 2>&1 || { tail gpurun_out/e_ts0_$s.log; exit 1; }
  grep -E "median|lanczos|iters" gpurun_out/e_ts0_$s.log
done
