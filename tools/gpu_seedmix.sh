#!/bin/bash
# In-flight scaling per seed mix: bench.py --seeds S --inflight P for each "P:S" argument (short runs).
#   gpurun -- 'bash tools/gpu_seedmix.sh 4:41,235,35 6:41,235,35 4:23 6:23'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/seedmix.log
: > $L
for spec in "$@"; do
  P=${spec%%:*}; S=${spec#*:}
  n=$(echo $S | tr ',' '\n' | wc -l)
  timeout -k 10 400 python bench.py --steps $n --warmup 1 --no-cpu-baseline --no-roofline --no-solo --seeds $S \
    --inflight $P --threads 1 --detail "" > gpurun_out/sm_line.json 2> gpurun_out/sm.err || { tail -5 gpurun_out/sm.err; exit 1; }
  python -c "import json; l=json.load(open('gpurun_out/sm_line.json')); print('p${P}t1 seeds ${S}', round(l['value'],4), round(l['sec_per_iter_per_seed_median_inflight'],3))" >> $L
  tail -1 $L
done
