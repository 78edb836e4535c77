set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
DT_RANKS=1 timeout -k 10 300 python -u tools/decision_trace.py dev graphm graphm_3 256 2 3 > gpurun_out/h_dev_ranks.jsonl 2> gpurun_out/h_dev_ranks.err || { tail gpurun_out/h_dev_ranks.err; exit 1; }
TTK_FUSED_MFMA=0 timeout -k 10 300 python -u tools/decision_trace.py dev graphm graphm_3 256 2 3 > gpurun_out/h_dev_nomfma.jsonl 2> gpurun_out/h_dev_nomfma.err || { tail gpurun_out/h_dev_nomfma.err; exit 1; }
TTK_SPLITK_MINK=100000 timeout -k 10 300 python -u tools/decision_trace.py dev graphm graphm_3 256 2 3 > gpurun_out/h_dev_nosplitk.jsonl 2> gpurun_out/h_dev_nosplitk.err || { tail gpurun_out/h_dev_nosplitk.err; exit 1; }
grep -c '^{' gpurun_out/h_dev_*.jsonl
