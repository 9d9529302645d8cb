#!/bin/bash
# round 4: hub_group_kernel phase cycles (MR_STAMPS build) on c2 and a single query
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/group_stamps.log; : > $L
export MR_LIB_PATH=marshrutka_amd/lib/variants/stamps/libmarshrutka_pf.so
for g in 16 8; do
MR_HUB_GROUP=$g timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
MR_HUB_GROUP=$g timeout -k 10 120 python -u tools/probes/group_time.py 15 1 4 15 >> $L 2>&1 || exit 1
done
