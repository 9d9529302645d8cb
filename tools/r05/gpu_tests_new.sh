#!/bin/bash
# round 5: the new lane/group-kernel parity tests, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_full_scale.py -k "c4" tests/test_gpu_parity.py::test_c2_full_batch_group_kernel \
  > gpurun_out/tests_new.log 2>&1 || { tail -50 gpurun_out/tests_new.log; exit 1; }
tail -15 gpurun_out/tests_new.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
