#!/bin/bash
# Same-box A/B: process count with the dgecon side stream on (default), and an eagerly created side
# stream (every process gets its second stream at context creation)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
common="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-solo"
run() {
  tag=$1; shift
  echo "== $tag $* $(date +%T)"
  timeout -k 10 300 env "$@" > gpurun_out/ab_${tag}.json 2> gpurun_out/ab_${tag}.err || { tail -5 gpurun_out/ab_${tag}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_${tag}.json'));print('$tag', round(d['value'],4), sorted([(r['seed'],round(r['runtime'],2)) for r in d['per_seed']]))"
}
echo "== lu $(date +%T)"
timeout -k 10 200 python tools/bench_lu.py > gpurun_out/lu_bench3.log 2>&1 || { tail -5 gpurun_out/lu_bench3.log; exit 1; }
cat gpurun_out/lu_bench3.log | grep -v amdgpu.ids
echo "== svd cases $(date +%T)"
timeout -k 10 200 python tools/bench_svd_cases.py ".svd_cases/*.npy" > gpurun_out/svd_cases3.log 2>&1 || { tail -5 gpurun_out/svd_cases3.log; exit 1; }
grep -A1 "svd_in_1.npy\|svd_in_9.npy" gpurun_out/svd_cases3.log
run p4 python bench.py $common --inflight 4
python3 -c "import json;d=json.load(open('gpurun_out/ab_p4.json'));print(sorted(set((r['seed'],r['num_iters'],r['gap']) for r in d['per_seed'])))"
run p4e TTK_EAGER_SIDE=1 python bench.py $common --inflight 4
run p6 python bench.py $common --inflight 6
run p6e TTK_EAGER_SIDE=1 python bench.py $common --inflight 6
run p8e TTK_EAGER_SIDE=1 python bench.py $common --inflight 8
echo "== done $(date +%T)"
