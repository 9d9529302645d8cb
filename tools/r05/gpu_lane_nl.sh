#!/bin/bash
# Fleetfoot on the lane kernel: parity (hub and lane), the lane modes, then the rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_scale.py tests/test_gpu_cert.py -x -q --timeout 300 --timeout-method thread \
  -k "fleetfoot or lanenl or (lane and golden) or certificate or cert or c4" > gpurun_out/tests_lane_nl.log 2>&1 || { tail -40 gpurun_out/tests_lane_nl.log; exit 1; }
tail -3 gpurun_out/tests_lane_nl.log
true
true
timeout -k 10 300 python -u tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_nl.log 2>&1 || { tail -20 gpurun_out/ff_rates_nl.log; exit 1; }
grep -v "ff=0" gpurun_out/ff_rates_nl.log
