set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/launch_sites.py maxcut maxcut_10 41 1 3 > gpurun_out/f_launch_sites_s41.txt 2>&1 || { tail gpurun_out/f_launch_sites_s41.txt; exit 1; }
head -40 gpurun_out/f_launch_sites_s41.txt
timeout -k 10 600 python -u tools/parity_report.py > gpurun_out/f_parity_report.txt 2> gpurun_out/f_parity_report.err || { tail gpurun_out/f_parity_report.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/f_parity_report.txt'):
    d = json.loads(l); print(d['key'], d['iters'], d.get('follows'), d['policy'][:120])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/f_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/f_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/f_pytest_gpu.log
