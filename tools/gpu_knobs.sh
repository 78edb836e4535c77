#!/bin/bash
# Whole-job rate per env knob setting (bench.py p4t1, --steps 5, short form): one line per argument,
# a comma-separated VAR=VALUE list or "-" for the defaults.
#   gpurun -- 'bash tools/gpu_knobs.sh - TTK_SCHUR_ONE=0 TTK_ARNOLDI_ONE=0,TTK_SPLITK_FUSED=0'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/knobs.log
: > $L
for spec in "$@"; do
  if [ "$spec" = "-" ]; then envs=""; else envs=${spec//,/ }; fi
  env $envs timeout -k 10 400 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline --no-solo \
    --inflight ${KN_P:-4} --threads 1 --detail "" > gpurun_out/kn_line.json 2> gpurun_out/kn.err || { tail -5 gpurun_out/kn.err; exit 1; }
  python -c "import json; l=json.load(open('gpurun_out/kn_line.json')); print('p${KN_P:-4}t1 ${spec}', round(l['value'],4), round(l['sec_per_iter_per_seed_median_inflight'],3))" >> $L
  tail -1 $L
done
