#!/bin/bash
# Slot-thread / process mix experiment (round 3): the same two seeds under different in-flight layouts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
common="--seeds 41,235 --steps 2 --warmup 1 --no-cpu-baseline --no-roofline"
run() {
  tag=$1; shift
  echo "== $tag $* $(date +%T)"
  timeout -k 10 300 env "$@" > gpurun_out/slots_${tag}.json 2> gpurun_out/slots_${tag}.err || { tail -5 gpurun_out/slots_${tag}.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/slots_${tag}.json'));print('$tag', round(d['value'],4), [(r['seed'],round(r['runtime'],2)) for r in d['per_seed']], d.get('solo_per_seed') and [(r['seed'],round(r['runtime'],2)) for r in d['solo_per_seed']])"
}
run t1p1 python bench.py $common --threads 1 --inflight 1
run t1p1def TTIPM_SLOT_STREAM=default python bench.py $common --threads 1 --inflight 1 --no-solo
run t2p2 python bench.py $common --threads 2 --inflight 2 --no-solo
run t1p2 python bench.py $common --threads 1 --inflight 2 --no-solo
run t1p2def TTIPM_SLOT_STREAM=default python bench.py $common --threads 1 --inflight 2 --no-solo
run t2p4 python bench.py $common --threads 2 --inflight 4 --no-solo
echo "== done $(date +%T)"
