#!/bin/bash
# Same-box A/B of HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device memory: lower launch latency)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() {
  tag=$1; shift
  echo "== $tag $* $(date +%T)"
  timeout -k 10 300 env "$@" > gpurun_out/ka_${tag}.json 2> gpurun_out/ka_${tag}.err || { tail -5 gpurun_out/ka_${tag}.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ka_${tag}.json'));print('$tag', round(d['value'],4), d.get('solo_per_seed') and [(r['seed'],round(r['runtime'],3)) for r in d['solo_per_seed']]); print(' gaps', sorted(set((r['seed'],r['num_iters'],r['gap']) for r in d['per_seed'])))"
}
common="--steps 3 --warmup 1 --no-cpu-baseline --no-roofline"
run p4 python bench.py $common --inflight 4
run p4k HIP_FORCE_DEV_KERNARG=1 python bench.py $common --inflight 4
run p4b python bench.py $common --inflight 4
run p4kb HIP_FORCE_DEV_KERNARG=1 python bench.py $common --inflight 4
echo "== done $(date +%T)"
