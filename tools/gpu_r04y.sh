#!/bin/bash
# round 4: group kernel phase cycles with the read-off split (MR_STAMPS build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/group_stamps2.log; : > $L
export MR_LIB_PATH=marshrutka_amd/lib/variants/stamps/libmarshrutka_pf.so
MR_HUB_GROUP=16 timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
timeout -k 10 120 python -u tools/probes/group_time.py 15 1 4 15 >> $L 2>&1 || exit 1
MR_HUB_GROUP=16 timeout -k 10 120 python -u tools/probes/group_time.py 65 1000 4 2024 >> $L 2>&1 || exit 1
