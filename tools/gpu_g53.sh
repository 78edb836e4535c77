set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/g53_gemm.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/g53_pytest.log 2>&1
