#!/bin/bash
# round 4: group kernel relax skip: parity (group modes), c2 and c1 bench lines with end to end
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "group or auto or c2_full or lane_kernel_selection" > gpurun_out/t_parity_r04zf.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 5 > gpurun_out/b_c2_zf.json 2> gpurun_out/b_c2_zf.err || exit 1
MR_TIMING=1 timeout -k 10 120 python bench.py --workload c1 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 20 > gpurun_out/b_c1_zf.json 2> gpurun_out/b_c1_zf.err
