#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 1100 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu tests/test_gpu_full_scale.py \
  -k "handed_over or fleetfoot_time_first" > gpurun_out/r06/tests_c4map.log 2>&1 || { tail -60 gpurun_out/r06/tests_c4map.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r06/tests_c4map.log | tail -12
