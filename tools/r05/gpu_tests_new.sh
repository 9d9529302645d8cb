#!/bin/bash
# round 5: the new parity tests (lane / group kernels at configs[3] / [1], the device
# region table), then the default bench line and c5's
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_region_table.py tests/test_gpu_full_scale.py -k "region or c4" \
  tests/test_gpu_parity.py::test_c2_full_batch_group_kernel \
  > gpurun_out/tests_new.log 2>&1 || { tail -60 gpurun_out/tests_new.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/tests_new.log | tail -20
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err || { tail -30 gpurun_out/bench_c5.err; exit 1; }
cat gpurun_out/bench_c5.json
