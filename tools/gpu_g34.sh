set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 2 4 8; do TTK_TRI_ROWS=$r timeout -k 10 200 python -u tools/bench_eig.py > gpurun_out/g34_eig_$r.log 2>&1 || exit 1; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x --timeout 120 --timeout-method thread -k "syev" > gpurun_out/g34_pytest.log 2>&1
