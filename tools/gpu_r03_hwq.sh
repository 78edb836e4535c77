#!/bin/bash
# Same-box A/B of HIP's hardware queues per process (GPU_MAX_HW_QUEUES, default 4) against the number
# of solve processes per GPU
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
common="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-solo"
run() {
  tag=$1; shift
  echo "== $tag $* $(date +%T)"
  timeout -k 10 300 env "$@" > gpurun_out/hwq_${tag}.json 2> gpurun_out/hwq_${tag}.err || { tail -5 gpurun_out/hwq_${tag}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/hwq_${tag}.json'));print('$tag', round(d['value'],4), sorted([(r['seed'],round(r['runtime'],2)) for r in d['per_seed']]))"
}
run p4 python bench.py $common --inflight 4
run p4q1 GPU_MAX_HW_QUEUES=1 python bench.py $common --inflight 4
run p6q1 GPU_MAX_HW_QUEUES=1 python bench.py $common --inflight 6
run p8q1 GPU_MAX_HW_QUEUES=1 python bench.py $common --inflight 8
run p6q2 GPU_MAX_HW_QUEUES=2 python bench.py $common --inflight 6
echo "== done $(date +%T)"
