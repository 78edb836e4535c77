set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for s in 14 35; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/p_s$s -o run -- python3 tools/time_solves.py maxcut maxcut_10 $s 1 1 > gpurun_out/p_s$s.log 2>&1 || { tail -20 gpurun_out/p_s$s.log; exit 1; }
  for f in $(find /tmp/p_s$s -name "*kernel_stats.csv"); do cp $f gpurun_out/p_mc10_s${s}_kernel_stats.csv; done
  grep median gpurun_out/p_s$s.log
done
timeout -k 10 300 python -u tools/profile_case.py maxcut maxcut_10 14 1 > gpurun_out/p_cprof_s14.log 2>&1 || { tail gpurun_out/p_cprof_s14.log; exit 1; }
ls gpurun_out | grep "^p_"
