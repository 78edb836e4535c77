#!/bin/bash
# After the 4-loads-in-flight staging of the VALU apply rows: phase split, the fused-apply and Schur
# kernel tests, and the bench's per-seed gaps (bit-identity against the committed line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for seed in 14 41; do
  echo "== seed $seed $(date +%T)"
  TTK_LIB_PATH=tools/micro/libttk_vprof.so timeout -k 10 200 python tools/mfma_phases.py maxcut maxcut_10 $seed 1 5 2>&1 | grep -v amdgpu.ids | tail -1
done
echo "== kernel tests $(date +%T)"
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stage_kt.log 2>&1 || { tail -20 gpurun_out/stage_kt.log; exit 1; }
tail -1 gpurun_out/stage_kt.log
echo "== bench $(date +%T)"
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/stage_bench.json 2> gpurun_out/stage_bench.err || { tail -5 gpurun_out/stage_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/stage_bench.json'));print(round(d['value'],4), d['solo_median_seed_s_per_iter'], [(r['seed'],round(r['runtime'],3)) for r in d['solo_per_seed']]); print(sorted(set((r['seed'],r['num_iters'],r['gap']) for r in d['per_seed'])))"
echo "== done $(date +%T)"
