set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g45_pytest.log 2>&1 && \
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/g45_b5.json 2>/dev/null
