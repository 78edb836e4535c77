#!/bin/bash
# VALU apply-row phase split (diagnostics build -DTTK_VALU_PROFILE) on maxcut_10 seeds 14 and 41,
# first 5 Newton systems each, with the default (side-by-side) and sequential Schur task terms
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for seed in 14 41; do
  for dual in 1 0; do
    echo "== seed $seed dual $dual $(date +%T)"
    TTK_APPLY_DUAL=$dual TTK_LIB_PATH=tools/micro/libttk_vprof.so timeout -k 10 200 python tools/mfma_phases.py maxcut maxcut_10 $seed 1 5 2>&1 | grep -v amdgpu.ids | tail -2
  done
done
echo "== done $(date +%T)"
