#!/bin/bash
# round 4 (late): profiles of the new default paths: c4 (lane kernel) and c2 (group kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/profile_round.sh r04b "c4 c2" > gpurun_out/prof_r04b.log 2>&1 || exit 1
bash tools/gpu_sq_wait.sh c4 gpurun_out/prof_r04b/sqw_c4
