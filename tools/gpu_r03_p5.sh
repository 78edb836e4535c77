#!/bin/bash
# Same-box A/B: 4 vs 5 solve processes per GPU (whole job over the five maxcut_10 seeds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
common="--steps 5 --warmup 1 --no-cpu-baseline --no-roofline --no-solo"
for p in 4 5 4 5; do
  echo "== p$p $(date +%T)"
  timeout -k 10 300 python bench.py $common --inflight $p > gpurun_out/p5_$p.json 2> gpurun_out/p5_$p.err || { tail -5 gpurun_out/p5_$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/p5_$p.json'));print('p$p', round(d['value'],4), d['config']['total_ipm_iters'], round(d['ms_per_step']*d['steps']/1e3,1))"
done
echo "== done $(date +%T)"
