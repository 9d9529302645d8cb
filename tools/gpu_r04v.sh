#!/bin/bash
# round 4: wave states of hub_group_kernel (G = 16) on c2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
MR_HUB_GROUP=16 bash tools/gpu_sq_wait.sh c2 gpurun_out/sqw_c2g16b && MR_HUB_GROUP=16 bash tools/gpu_sq.sh c2 gpurun_out/sq_c2g16b
