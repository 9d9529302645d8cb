#!/bin/bash
# round 4: hub_group_kernel (one source per 8 / 16 lanes) — parity in the group modes, c2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/group_min > gpurun_out/group_min.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    -k "group or lane_kernel_selection or c2_full or default_params" > gpurun_out/t_group.log 2>&1 &&
timeout -k 10 120 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 3 > gpurun_out/b_c2_g8.json 2> gpurun_out/b_c2_g8.err &&
MR_HUB_GROUP=16 timeout -k 10 120 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 3 > gpurun_out/b_c2_g16.json 2> gpurun_out/b_c2_g16.err &&
MR_HUB_GROUP=0 timeout -k 10 120 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 3 > gpurun_out/b_c2_hub.json 2> gpurun_out/b_c2_hub.err
