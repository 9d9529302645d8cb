#!/bin/bash
# round 5 baseline probes: host phase timings of a fresh batch (MR_TIMING) at 1M and
# 125k, the Fleetfoot rates at 1025^2 / 125k, and a kernel trace of the default bench
set -o pipefail
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
MR_TIMING=1 timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --e2e-reps 3 > gpurun_out/probe/e2e_1m.json 2> gpurun_out/probe/e2e_1m.err || exit 1
MR_TIMING=1 timeout -k 10 300 python bench.py --steps 5 --queries 125000 --no-cpu-baseline --e2e-reps 3 > gpurun_out/probe/e2e_125k.json 2> gpurun_out/probe/e2e_125k.err || exit 1
grep MR_TIMING gpurun_out/probe/e2e_1m.err | tail -12
grep MR_TIMING gpurun_out/probe/e2e_125k.err | tail -12
timeout -k 10 400 python tools/ff_rates.py 1025 125000 3 > gpurun_out/probe/ff_rates.log 2>&1 || exit 1
cat gpurun_out/probe/ff_rates.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe/kt_c4 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 0 > gpurun_out/probe/kt_c4.log 2>&1 || exit 1
tail -1 gpurun_out/probe/kt_c4.log
