#!/bin/bash
# In-flight layouts against the HW queue budget per process (GPU_MAX_HW_QUEUES): one bench line per
# "PROCS:QUEUES" argument (QUEUES "-" = the default; TTIPM_HW_QUEUES sets GPU_MAX_HW_QUEUES), short runs, value + per-seed in-flight s/iter.
#   gpurun -- 'bash tools/gpu_hwq.sh 4:- 4:1 6:1'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/hwq.log
: > $L
for spec in "$@"; do
  P=${spec%%:*}; Q=${spec#*:}
  if [ "$Q" = "-" ]; then envq=""; else envq="TTIPM_HW_QUEUES=$Q"; fi
  env $envq timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-solo \
    --inflight $P --threads 1 --detail "" > gpurun_out/hwq_line.json 2> gpurun_out/hwq.err || { tail -5 gpurun_out/hwq.err; exit 1; }
  python -c "import json,sys; l=json.load(open('gpurun_out/hwq_line.json')); print('p${P}t1 queues=${Q}', round(l['value'],4), round(l['sec_per_iter_per_seed_median_inflight'],3))" >> $L
  tail -1 $L
done
