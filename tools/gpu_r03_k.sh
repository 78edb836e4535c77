set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "split or fused_apply_mfma or env_update_mfma" --timeout 300 --timeout-method thread > gpurun_out/k_tests.log 2>&1 || { tail -30 gpurun_out/k_tests.log; exit 1; }
tail -2 gpurun_out/k_tests.log
for cs in 0 1; do
  TTK_MFMA_CSPLIT=$cs timeout -k 10 400 python bench.py --config configs/graphm_3.yaml --rank 2 --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline > gpurun_out/k_graphm_cs$cs.json 2> gpurun_out/k_graphm_cs$cs.err || { tail gpurun_out/k_graphm_cs$cs.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/k_graphm_cs$cs.json').read().strip().splitlines()[-1])
print('csplit $cs', d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['per_seed'][0]['num_iters'], d['per_seed'][0]['gap'])"
done
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k_stats -o run -- python3 bench.py --config configs/graphm_3.yaml --rank 2 --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline > gpurun_out/k_stats.log 2>&1 || { tail -20 gpurun_out/k_stats.log; exit 1; }
for f in $(find /tmp/k_stats -name "*stats.csv"); do cp $f gpurun_out/k_graphm_$(basename $f); done
ls gpurun_out | grep k_graphm
