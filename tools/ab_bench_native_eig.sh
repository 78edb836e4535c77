# Whole-job bench with the native eigen-ALS on and off, alternating (A/B on one box).
#   bash tools/ab_bench_native_eig.sh [extra bench.py args, e.g. --threads 2 --inflight 4]
set -o pipefail
for i in 1 2; do
  for nat in 1 0; do
    TTIPM_NATIVE_EIG=$nat timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline --no-solo --detail '' "$@" > gpurun_out/ab_bench_n${nat}_$i.json 2> gpurun_out/ab_bench_n${nat}_$i.err || exit 1
    echo "native=$nat rep $i: $(python -c "import json;d=json.load(open('gpurun_out/ab_bench_n${nat}_$i.json'));print(d['value'], d['ms_per_step'], d['config']['workload'])")"
  done
done
