#!/bin/bash
# the lane kernel's count order, busiest sources first (default) or last (MR_LANE_ORDER=asc)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_dev_group.py tests/test_gpu_full_scale.py -k "dev_group or device_grouping or c4_full or c4_lane" -x -q --timeout 400 --timeout-method thread > gpurun_out/r06/order_dir_tests.log 2>&1 || { tail -30 gpurun_out/r06/order_dir_tests.log; exit 1; }
tail -1 gpurun_out/r06/order_dir_tests.log
for o in desc asc desc asc; do
  for q in 1000000 125000; do
    MR_LANE_ORDER=$o timeout -k 10 200 python -u bench.py --workload c4 --queries $q --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/order_${o}_$q.log 2>&1 || { tail -20 gpurun_out/r06/order_${o}_$q.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/r06/order_${o}_$q.log').read().strip().splitlines()[-1]); print('$o $q', d['ms_per_step'], d['roofline']['kernel_ms'])"
  done
done
