#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_scale.py -k "lane or c4_full" -x -q --timeout 400 --timeout-method thread > gpurun_out/r06/qpf_tests.log 2>&1 || { tail -40 gpurun_out/r06/qpf_tests.log; exit 1; }
tail -1 gpurun_out/r06/qpf_tests.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/bench_c4_qpf.log 2>&1 || { tail -20 gpurun_out/r06/bench_c4_qpf.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r06/bench_c4_qpf.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['kernel_ms'], d['value'])"
FRESH=1 MR_TIMING=1 timeout -k 10 300 python -u tools/r06/fetch_time.py > gpurun_out/r06/fetch_time_fresh.log 2>&1 || { tail -20 gpurun_out/r06/fetch_time_fresh.log; exit 1; }
grep -v "MR_TIMING plan\|MR_TIMING run" gpurun_out/r06/fetch_time_fresh.log | tail -30
