#!/bin/bash
# round 4: group kernel destinations phase experiments (256: no boundary loop, 512: no emission)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/group_time7.log; : > $L
for f in 0 256 512 768 32; do
  MR_HUB_GROUP=16 MR_DBG_FLAGS=$f timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
for f in 0 256 512 768; do
  MR_DBG_FLAGS=$f timeout -k 10 120 python -u tools/probes/group_time.py 15 1 4 15 >> $L 2>&1 || exit 1
done
