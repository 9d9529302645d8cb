#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/group_time9.log; : > $L
for f in 0 128 512 640; do
  MR_HUB_GROUP=16 MR_DBG_FLAGS=$f timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
