#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests/test_gpu_dev_group.py tests/test_gpu_parity.py -k "group or c2 or dev_group or device_grouping" -x -q --timeout 400 --timeout-method thread > gpurun_out/r06/group_order_tests.log 2>&1 || { tail -40 gpurun_out/r06/group_order_tests.log; exit 1; }
tail -1 gpurun_out/r06/group_order_tests.log
for o in 0 1 0 1; do
  MR_GROUP_ORDER=$o timeout -k 10 300 python -u bench.py --workload c2 --steps 200 --warmup 10 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/bench_c2_go$o.log 2>&1 || { tail -20 gpurun_out/r06/bench_c2_go$o.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06/bench_c2_go$o.log').read().strip().splitlines()[-1])
print('order $o', d['ms_per_step'], d['roofline']['kernel_ms'], d['value'])"
done
set -o pipefail
mkdir -p gpurun_out/r06
for s in 2024 4096; do
  timeout -k 10 400 python -u tools/ff_rates.py 1025 125000 3 $s > gpurun_out/r06/ff_rates_$s.log 2>&1 || { tail -20 gpurun_out/r06/ff_rates_$s.log; exit 1; }
  grep "sort=(1" gpurun_out/r06/ff_rates_$s.log
done
timeout -k 10 300 python -u tools/r06/ff_c4map.py 4096 > gpurun_out/r06/ff_c4map.log 2>&1 || { tail -20 gpurun_out/r06/ff_c4map.log; exit 1; }
cat gpurun_out/r06/ff_c4map.log
