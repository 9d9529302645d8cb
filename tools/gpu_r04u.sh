#!/bin/bash
# round 4: host-built lane/group LDS block, group prefetch: parity, timings, c2/c4 bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t_parity_r04u.log 2>&1 || exit 1
L=gpurun_out/group_time5.log; : > $L
for env in "MR_HUB_GROUP=8" "MR_HUB_GROUP=16" "MR_HUB_GROUP=32" "MR_HUB_GROUP=16 MR_DBG_FLAGS=32" "MR_HUB_GROUP=16 MR_DBG_FLAGS=128"; do
  env $env timeout -k 10 120 python -u tools/probes/group_time.py >> $L 2>&1 || exit 1
done
for env in "MR_HUB_GROUP=16" "MR_HUB_GROUP=32" "MR_HUB_GROUP=0"; do
  env $env timeout -k 10 120 python -u tools/probes/group_time.py 15 1 4 15 >> $L 2>&1 || exit 1
done
for g in 16 32; do
MR_HUB_GROUP=$g timeout -k 10 120 python bench.py --workload c2 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 3 > gpurun_out/b_c2_g$g.json 2> gpurun_out/b_c2_g$g.err || exit 1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > gpurun_out/b_c4_blob.json 2> gpurun_out/b_c4_blob.err
