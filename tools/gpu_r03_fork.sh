#!/bin/bash
# Same-box A/B of the in-flight process count and of the dgecon side stream (TTK_LU_FORK)
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
echo "== latency micro $(date +%T)"
(cd tools/micro && timeout -k 10 120 hipcc -O3 --offload-arch=gfx950 latency.hip -o /tmp/latency_bin) && timeout -k 10 60 /tmp/latency_bin > gpurun_out/latency_micro.log 2>&1 || { tail -5 gpurun_out/latency_micro.log; exit 1; }
cat gpurun_out/latency_micro.log
echo "== svd cases $(date +%T)"
timeout -k 10 200 python tools/bench_svd_cases.py ".svd_cases/*.npy" > gpurun_out/svd_cases2.log 2>&1 || { tail -5 gpurun_out/svd_cases2.log; exit 1; }
grep -A1 "svd_in_1.npy\|svd_in_9.npy" gpurun_out/svd_cases2.log
run p4 python bench.py $common --inflight 4
run p4f0 TTK_LU_FORK=0 python bench.py $common --inflight 4
run p6f0 TTK_LU_FORK=0 python bench.py $common --inflight 6
run p4b python bench.py $common --inflight 4
echo "== done $(date +%T)"
