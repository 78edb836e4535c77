set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mw in 16384 65536 262144; do
  for s in 14 41 35; do
    TTK_LGMRES_MW_MIN=$mw timeout -k 10 300 python tools/time_solves.py maxcut maxcut_10 $s 1 2 > gpurun_out/q_ts_${mw}_$s.log 2>&1 || { tail gpurun_out/q_ts_${mw}_$s.log; exit 1; }
    echo "mw=$mw s=$s $(grep median gpurun_out/q_ts_${mw}_$s.log)"
  done
done
