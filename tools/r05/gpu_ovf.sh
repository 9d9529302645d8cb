#!/bin/bash
# round 5: overflow pool in record order (bound outputs), the overflow tests, the N>1 record gather
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "overflow" > gpurun_out/tests_ovf.log 2>&1 || { tail -60 gpurun_out/tests_ovf.log; exit 1; }
grep -cE "PASSED" gpurun_out/tests_ovf.log; tail -2 gpurun_out/tests_ovf.log
