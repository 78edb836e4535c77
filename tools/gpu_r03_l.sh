set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export TTK_SPLITK_MINK=128
timeout -k 10 400 python bench.py --config configs/graphm_3.yaml --rank 2 --steps 1 --warmup 0 --inflight 1 --no-cpu-baseline > gpurun_out/l_graphm_mink128.json 2> gpurun_out/l_graphm_mink128.err || { tail gpurun_out/l_graphm_mink128.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/l_graphm_mink128.json').read().strip().splitlines()[-1])
print('mink128', d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['per_seed'][0]['num_iters'], d['per_seed'][0]['gap'])"
timeout -k 10 300 python -u tools/decision_trace.py dev graphm graphm_3 256 2 4 > gpurun_out/l_dev_mink128.jsonl 2> gpurun_out/l_dev_mink128.err || { tail gpurun_out/l_dev_mink128.err; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -k "bounded_trace or maxcut_12" --timeout 300 --timeout-method thread > gpurun_out/l_tests.log 2>&1 || { tail -30 gpurun_out/l_tests.log; exit 1; }
tail -2 gpurun_out/l_tests.log
