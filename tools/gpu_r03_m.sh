set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
export TTK_SPLITK_MINK=${MINK:-128}
timeout -k 10 900 python -u tools/parity_report.py > gpurun_out/m_parity_report.txt 2> gpurun_out/m_parity_report.err || { tail gpurun_out/m_parity_report.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/m_parity_report.txt'):
    if l.startswith('{'):
        d = json.loads(l); print(d['key'], d['iters'], d.get('follows'), d['policy'][:150])"
timeout -k 10 300 python -u tools/parity_report.py maxcut_12_r2_s80 > gpurun_out/m_parity_m12.txt 2> gpurun_out/m_parity_m12.err || { tail gpurun_out/m_parity_m12.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/m_parity_m12.txt'):
    if l.startswith('{'):
        d = json.loads(l); print(d['key'], d['iters'], d.get('follows'), d['policy'][:300])"
