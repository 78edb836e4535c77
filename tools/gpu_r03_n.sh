set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mk in 256 128; do
  echo "== TTK_SPLITK_MINK=$mk"
  TTK_SPLITK_MINK=$mk timeout -k 10 300 python tools/bench_gemm.py > gpurun_out/n_gemm_mink$mk.txt 2>&1 || { tail gpurun_out/n_gemm_mink$mk.txt; exit 1; }
  grep -E "^ *(212|116|216|60|192|56) " gpurun_out/n_gemm_mink$mk.txt
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/n_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/n_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/n_pytest_gpu.log
timeout -k 10 900 python bench.py > gpurun_out/n_bench.json 2> gpurun_out/n_bench.err || { tail gpurun_out/n_bench.err; exit 1; }
cut -c1-400 gpurun_out/n_bench.json
