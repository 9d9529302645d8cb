#!/bin/bash
# round 4: wave-state breakdown of hub_group_kernel on c2 (G = 8 and 16)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_sq_wait.sh c2 gpurun_out/sqw_c2g8 &&
MR_HUB_GROUP=16 bash tools/gpu_sq_wait.sh c2 gpurun_out/sqw_c2g16
