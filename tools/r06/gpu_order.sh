#!/bin/bash
# lane order by query count: grouping / parity tests, c4 bench, stamps
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests/test_gpu_dev_group.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -k "dev_group or device_grouping or lane or c2 or fetch or wire or golden or c4" -x -q --timeout 400 --timeout-method thread > gpurun_out/r06/order_tests.log 2>&1 || { tail -40 gpurun_out/r06/order_tests.log; exit 1; }
tail -1 gpurun_out/r06/order_tests.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r06/bench_c4_order.log 2>&1 || { tail -20 gpurun_out/r06/bench_c4_order.log; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r06/bench_c4_order.log').read().strip().splitlines()[-1])
print(d['ms_per_step'], d['roofline']['kernel_ms'], d['value'])
for k in ('end_to_end','end_to_end_pinned'): print(k, {x: round(d[k][x],3) for x in ('e2e_queries_per_s','ms','plan_create_ms','run_ms','fetch_ms')})"
MR_LIB_PATH=marshrutka_amd/lib/diag/libmarshrutka_pf.so timeout -k 10 200 python -u bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/lane_stamps2.log 2>&1 || exit 1
grep "MR_STAMPS lane" gpurun_out/r06/lane_stamps2.log | tail -1
