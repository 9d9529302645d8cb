#!/bin/bash
# lane-kernel phase stamps on c4 (diagnostic build, MR_STAMPS)
set -o pipefail
mkdir -p gpurun_out/r06
MR_LIB_PATH=marshrutka_amd/lib/diag/libmarshrutka_pf.so timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/lane_stamps.log 2>&1 || { tail -20 gpurun_out/r06/lane_stamps.log; exit 1; }
grep "MR_STAMPS" gpurun_out/r06/lane_stamps.log | tail -4
