#!/bin/bash
# round 4: cooperative read-off in the group kernel: parity (all modes), timings, c2 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t_parity_r04za.log 2>&1 || exit 1
L=gpurun_out/group_time8.log; : > $L
for g in 16 32 8; do
  MR_HUB_GROUP=$g timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/probes/group_time.py 15 1 4 15 >> $L 2>&1 || exit 1
timeout -k 10 120 python bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 3 > gpurun_out/b_c2_coop.json 2> gpurun_out/b_c2_coop.err
