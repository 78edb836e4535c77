#!/bin/bash
# Round-3 validation + A/B in one call: LU / SVD kernel timings, bench gaps (bit-identity against the
# committed line), VALU thread count, process count with / without an eager side stream
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
echo "== lu $(date +%T)"
timeout -k 10 200 python tools/bench_lu.py > gpurun_out/lu_bench3.log 2>&1 || { tail -5 gpurun_out/lu_bench3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/lu_bench3.log
echo "== svd cases $(date +%T)"
timeout -k 10 200 python tools/bench_svd_cases.py ".svd_cases/*.npy" > gpurun_out/svd_cases3.log 2>&1 || { tail -5 gpurun_out/svd_cases3.log; exit 1; }
grep -A1 "svd_in_1.npy\|svd_in_9.npy" gpurun_out/svd_cases3.log
run() {
  tag=$1; shift
  echo "== $tag $* $(date +%T)"
  timeout -k 10 300 env "$@" > gpurun_out/ab_${tag}.json 2> gpurun_out/ab_${tag}.err || { tail -5 gpurun_out/ab_${tag}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_${tag}.json'));print('$tag', round(d['value'],4), sorted([(r['seed'],round(r['runtime'],2)) for r in d['per_seed']]), d.get('solo_per_seed') and [(r['seed'],round(r['runtime'],3)) for r in d['solo_per_seed']]); print(' gaps', sorted(set((r['seed'],r['num_iters'],r['gap']) for r in d['per_seed'])))"
}
common="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-solo"
run p4 python bench.py $common --inflight 4
solo="--seeds 14,35 --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline --no-roofline"
run v256 TTK_VALU_THREADS=256 python bench.py $solo
run v512 TTK_VALU_THREADS=512 python bench.py $solo
run v1024 TTK_VALU_THREADS=1024 python bench.py $solo
run p4e TTK_EAGER_SIDE=1 python bench.py $common --inflight 4
run p6 python bench.py $common --inflight 6
run p6e TTK_EAGER_SIDE=1 python bench.py $common --inflight 6
echo "== done $(date +%T)"
