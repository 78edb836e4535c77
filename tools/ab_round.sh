#!/bin/bash
# ttk_round before/after on one box: the previous library (ab/libttk_head.so) and the working
# tree's, alternating; the kernel dump of both compared bit for bit; the rounding / dense-solve
# parity tests and the QR kernel tests; an s41 solve pair on each.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for lib in ab/libttk_head.so tensor-train-interior-point-method_amd/libttk.so; do
    echo "== $lib ($i)"
    TTK_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 -u tools/bench_round.py 300 || exit $?
  done
done
TTK_LIB_PATH=$PWD/ab/libttk_head.so timeout -k 10 180 python3 -u tools/dump_kernels.py gpurun_out/dump_a.npz > /dev/null || exit $?
timeout -k 10 180 python3 -u tools/dump_kernels.py gpurun_out/dump_b.npz > /dev/null || exit $?
python3 tools/cmp_dump.py gpurun_out/dump_a.npz gpurun_out/dump_b.npz
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_abi.py "tests/test_gpu_kernels.py" -k "round or schur or zipup or qr or abi" || exit $?
for i in 1 2; do
  for lib in ab/libttk_head.so tensor-train-interior-point-method_amd/libttk.so; do
    echo "== s41 $lib ($i)"
    TTK_LIB_PATH=$PWD/$lib timeout -k 10 120 python3 -u tools/solve_twice.py maxcut maxcut_10 41 1 2>&1 | grep -E "Convergence in|first" || exit $?
  done
done
