#!/bin/bash
# round 4: where hub_group_kernel's time goes on c2 (experiment bits), G = 8 / 16, and hub_kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/group_time.log; : > $L
for env in "MR_HUB_GROUP=8" "MR_HUB_GROUP=16" "MR_HUB_GROUP=0" "MR_HUB_GROUP=8 MR_DBG_FLAGS=64" "MR_HUB_GROUP=8 MR_DBG_FLAGS=32" "MR_HUB_GROUP=8 MR_DBG_FLAGS=96" "MR_HUB_GROUP=16 MR_DBG_FLAGS=96"; do
  env $env timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
for env in "MR_HUB_GROUP=8" "MR_HUB_GROUP=0"; do
  env $env timeout -k 10 120 python -u tools/probes/group_time.py 15 1 4 15 >> $L 2>&1 || exit 1
  env $env timeout -k 10 120 python -u tools/probes/group_time.py 65 100 4 2024 >> $L 2>&1 || exit 1
done
bash tools/gpu_sq.sh c2 gpurun_out/sq_c2g
