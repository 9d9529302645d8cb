#!/bin/bash
# round 4: hub_group_kernel on c2 without the exact-tie list compares (timing only)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/group_time2.log; : > $L
for env in "MR_HUB_GROUP=16" "MR_HUB_GROUP=16 MR_DBG_FLAGS=128" "MR_HUB_GROUP=8 MR_DBG_FLAGS=128" "MR_HUB_GROUP=16 MR_DBG_FLAGS=160"; do
  env $env timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
