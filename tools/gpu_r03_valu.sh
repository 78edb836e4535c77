#!/bin/bash
# Same-box A/B of the VALU apply-row thread count (TTK_VALU_THREADS; results unchanged by construction):
# one-at-a-time solves of maxcut_10 seeds 14 and 35 (LGMRES-heavy) and their final gaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
common="--seeds 14,35 --steps 1 --warmup 1 --inflight 1 --no-cpu-baseline --no-roofline"
for t in 256 512 1024 256; do
  echo "== valu $t $(date +%T)"
  TTK_VALU_THREADS=$t timeout -k 10 300 python bench.py $common > gpurun_out/valu_$t.json 2> gpurun_out/valu_$t.err || { tail -5 gpurun_out/valu_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/valu_$t.json'));print('valu $t', [(r['seed'],round(r['runtime'],3),r['gap']) for r in d['solo_per_seed']], [(r['seed'],round(r['runtime'],3)) for r in d['per_seed']])"
done
echo "== done $(date +%T)"
