# Whole-job bench under bit-identical knob variants, alternating with the defaults on one box.
#   bash tools/ab_knobs.sh "TTK_SPLITK_FUSED=0" "TTK_ARNOLDI_ONE=0" ...   [BENCH_ARGS env: extra bench.py args;
#   SOLO=" " also runs the one-solve-at-a-time pass (per-seed median)]
set -o pipefail
for i in 1 2; do
  for v in "DEFAULT=1" "$@"; do
    tag=$(echo "$v" | tr '=' '_')
    env "$v" timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-roofline ${SOLO:---no-solo} --detail '' $BENCH_ARGS > gpurun_out/abk_${tag}_$i.json 2> gpurun_out/abk_${tag}_$i.err || exit 1
    echo "$v rep $i: $(python -c "import json;d=json.load(open('gpurun_out/abk_${tag}_$i.json'));print(d['value'], d['ms_per_step'], d.get('sec_per_iter_per_seed_median'))")"
  done
done
