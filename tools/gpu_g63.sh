set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -rs --timeout 300 --timeout-method thread > gpurun_out/g63_pytest.log 2>&1
