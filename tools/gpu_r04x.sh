#!/bin/bash
# round 4: group kernel emission from precomputed tail commands: parity (group modes), timings, phase cycles
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "group or auto or c2_full or lane_kernel_selection" > gpurun_out/t_parity_r04x.log 2>&1 || exit 1
L=gpurun_out/group_time6.log; : > $L
for env in "MR_HUB_GROUP=16" "MR_HUB_GROUP=32" "MR_HUB_GROUP=16 MR_DBG_FLAGS=32"; do
  env $env timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/probes/group_time.py 15 1 4 15 >> $L 2>&1 || exit 1
MR_LIB_PATH=marshrutka_amd/lib/variants/stamps/libmarshrutka_pf.so MR_HUB_GROUP=16 timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 3 > gpurun_out/b_c2_ct.json 2> gpurun_out/b_c2_ct.err
