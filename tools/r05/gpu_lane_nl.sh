#!/bin/bash
# Fleetfoot on the lane kernel: parity (hub and lane), the lane modes, then the rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "fleetfoot_hub or lanenl or (lane and golden) or certificate_sfm" > gpurun_out/tests_lane_nl.log 2>&1 || { tail -40 gpurun_out/tests_lane_nl.log; exit 1; }
tail -3 gpurun_out/tests_lane_nl.log
timeout -k 10 300 python -u tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_nl.log 2>&1 || { tail -20 gpurun_out/ff_rates_nl.log; exit 1; }
cat gpurun_out/ff_rates_nl.log
MR_LANE_NONLIN=1 timeout -k 10 300 python -u tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_nl_all.log 2>&1 || { tail -20 gpurun_out/ff_rates_nl_all.log; exit 1; }
grep "sort=(1" gpurun_out/ff_rates_nl_all.log
