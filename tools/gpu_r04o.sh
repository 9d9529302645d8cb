#!/bin/bash
# round 4: hub_group_kernel diagnostics (group_min micro check, golden fixtures through the group kernel)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
ok() { case "$1" in 0|1) return 0 ;; *) echo "step failed with $1; stopping" ; exit "$1" ;; esac; }
timeout -k 10 60 ./tools/micro/group_min > gpurun_out/group_min.log 2>&1; ok $?
timeout -k 10 300 python -u tools/probes/group_dbg.py s15_mixed > gpurun_out/group_dbg.log 2>&1; ok $?
timeout -k 10 300 python -u tools/probes/group_dbg.py s5_all_sorts >> gpurun_out/group_dbg.log 2>&1; ok $?
