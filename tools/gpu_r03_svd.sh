#!/bin/bash
# SVD unfoldings of maxcut_10 seed 23 (p in [33, 96]) dumped from a real solve, then timed one by one
# with the one-workgroup kernel's phase split; then the bench with the dgecon estimate on the main stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
echo "== dump $(date +%T)"
TTIPM_DUMP_SVD=33 TTIPM_DUMP_SVD_MAX=96 timeout -k 10 200 python tools/run_case.py maxcut maxcut_10 23 1 > gpurun_out/svd_dump.log 2>&1 || { tail -5 gpurun_out/svd_dump.log; exit 1; }
echo "== cases $(date +%T)"
timeout -k 10 200 python tools/bench_svd_cases.py "gpurun_out/svd_in_*.npy" > gpurun_out/svd_cases.log 2>&1 || { tail -5 gpurun_out/svd_cases.log; exit 1; }
cat gpurun_out/svd_cases.log
echo "== bench fork0 $(date +%T)"
TTK_LU_FORK=0 timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/fork0_bench.json 2> gpurun_out/fork0_bench.err || { tail -5 gpurun_out/fork0_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/fork0_bench.json'));print('fork0', d['value'], d['solo_median_seed_s_per_iter'], [(r['seed'],round(r['runtime'],2)) for r in d['solo_per_seed']])"
echo "== done $(date +%T)"
