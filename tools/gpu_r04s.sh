#!/bin/bash
# round 4: hub_group_kernel after the prologue / LDS changes: group parity modes, then c2 timings
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "group or lane_kernel_selection or c2_full or lane-lds" > gpurun_out/t_group2.log 2>&1 || exit 1
L=gpurun_out/group_time3.log; : > $L
for env in "MR_HUB_GROUP=8" "MR_HUB_GROUP=16" "MR_HUB_GROUP=16 MR_DBG_FLAGS=128" "MR_HUB_GROUP=16 MR_DBG_FLAGS=32"; do
  env $env timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
