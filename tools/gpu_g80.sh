set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for s in 80 45 23 53 12 0 1 2; do
timeout -k 10 300 python -u tools/run_case.py maxcut maxcut_12 $s 2 2>&1 | grep -E "Convergence in|Convergence after" | tr '\n' ' ' >> gpurun_out/g80.log || exit 1
echo " <- seed $s" >> gpurun_out/g80.log
done
