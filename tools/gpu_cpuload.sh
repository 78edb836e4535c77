#!/bin/bash
# Is the in-flight wall between 4 and 6 solves the host CPU?  bench.py p4t1 alone, then with B
# CPU-only busy-loop processes beside it (no GPU use), then p6t1 alone.
#   gpurun -- 'bash tools/gpu_cpuload.sh 2 4'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/cpuload.log
: > $L
echo "affinity: $(python -c 'import os; print(sorted(os.sched_getaffinity(0)))')" >> $L
lscpu -e=CPU,CORE,SOCKET 2>/dev/null | awk 'NR==1 || $1 < 16 || ($1 >= 128 && $1 < 144)' >> $L || true
run() {  # $1 = label, $2 = inflight
  timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-solo \
    --inflight $2 --threads 1 --detail "" > gpurun_out/cl_line.json 2> gpurun_out/cl.err || { tail -5 gpurun_out/cl.err; return 1; }
  python -c "import json; l=json.load(open('gpurun_out/cl_line.json')); print('$1', round(l['value'],4), round(l['sec_per_iter_per_seed_median_inflight'],3))" >> $L
  tail -1 $L
}
run "p4t1" 4 || exit 1
for B in "$@"; do
  pids=""
  for i in $(seq 1 $B); do python -c "while True: pass" & pids="$pids $!"; done
  run "p4t1 + $B busy CPU processes" 4; rc=$?
  kill $pids; wait $pids 2>/dev/null
  [ $rc -eq 0 ] || exit 1
done
run "p6t1" 6 || exit 1
cat $L
