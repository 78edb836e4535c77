set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_run.sh r03pmc "pmc:FETCH_SIZE" "pmc:WRITE_SIZE" "stats" || exit 1
timeout -k 10 900 python -u tools/scan_seeds.py maxcut maxcut_12 2 7 40 > gpurun_out/r_scan_m12.txt 2>&1 || { tail gpurun_out/r_scan_m12.txt; exit 1; }
grep '^{' gpurun_out/r_scan_m12.txt
