#!/bin/bash
# kernel trace of the world-1 RCCL bench path (wire gather) on c4
set -o pipefail
mkdir -p gpurun_out/r06
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
MR_BENCH_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_dist1 -o run --output-format csv -- python3 bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/prof_dist1.log 2>&1 || { tail -30 gpurun_out/r06/prof_dist1.log; exit 1; }

f=$(find gpurun_out/r06/prof_dist1 -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/r06/dist1_kernel_stats.csv
