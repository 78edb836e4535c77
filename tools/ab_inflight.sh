# Whole-job bench over in-flight layouts and hardware-queue budgets, alternating on one box:
#   bash tools/ab_inflight.sh "4:8" "6:2" ...   (inflight:GPU_MAX_HW_QUEUES per process)
set -o pipefail
for i in 1 2; do
  for v in "$@"; do
    p=${v%%:*}; q=${v##*:}
    TTIPM_HW_QUEUES=$q timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-solo --detail '' --inflight $p > gpurun_out/abi_${p}_${q}_$i.json 2> gpurun_out/abi_${p}_${q}_$i.err || exit 1
    echo "inflight=$p queues=$q rep $i: $(python -c "import json;d=json.load(open('gpurun_out/abi_${p}_${q}_$i.json'));print(d['value'], d['ms_per_step'], d['config']['workload'])")"
  done
done
