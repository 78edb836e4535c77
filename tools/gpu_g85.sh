set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/g85_sweep.txt
: > $out
for cfg in "" "TTK_FUSED_MAX_FLOPS=1e7" "TTK_FUSED_MAX_FLOPS=1e6" "TTIPM_LGMRES_CHUNK=16" "TTIPM_LGMRES_CHUNK=4" "TTK_TRI_ROWS=8" "TTK_GEMM64_KS=8"; do
  echo "== $cfg" >> $out
  env $cfg timeout -k 10 200 python bench.py --steps 2 --warmup 1 > gpurun_out/g85_one.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/g85_one.log').read().strip().splitlines()[-1]);print(d['value'],[(s['num_iters'],s['gap']) for s in d['per_seed']])" >> $out
done
