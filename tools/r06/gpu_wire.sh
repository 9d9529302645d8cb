#!/bin/bash
# wire records: parity tests, the all-destinations test that failed in the suite, the
# world-1 RCCL bench path on c4 (wire gather)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_sssp.py tests/test_gpu_parity.py -k "wire or every_cell" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/wire_tests.log 2>&1 || { tail -60 gpurun_out/r06/wire_tests.log; exit 1; }
tail -3 gpurun_out/r06/wire_tests.log
MR_BENCH_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_PORT=29511 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/bench_c4_dist1.log 2>&1 || { tail -30 gpurun_out/r06/bench_c4_dist1.log; exit 1; }
tail -2 gpurun_out/r06/bench_c4_dist1.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 > gpurun_out/r06/bench_c4_plain.log 2>&1 || { tail -30 gpurun_out/r06/bench_c4_plain.log; exit 1; }
tail -1 gpurun_out/r06/bench_c4_plain.log
