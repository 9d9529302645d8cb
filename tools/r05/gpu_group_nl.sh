#!/bin/bash
# Fleetfoot on the group kernel: the Fleetfoot parity cases on every kernel, the group
# parity modes, then the c2-size rates
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
  -k "fleetfoot or group or lanenl" > gpurun_out/tests_group_nl.log 2>&1 || { tail -40 gpurun_out/tests_group_nl.log; exit 1; }
tail -n 3 gpurun_out/tests_group_nl.log
timeout -k 10 300 python -u tools/ff_rates.py 65 10000 5 > gpurun_out/ff_rates_c2.log 2>&1 || { tail -20 gpurun_out/ff_rates_c2.log; exit 1; }
cat gpurun_out/ff_rates_c2.log
MR_LANE_NONLIN=0 timeout -k 10 300 python -u tools/ff_rates.py 65 10000 5 > gpurun_out/ff_rates_c2_hub.log 2>&1 || { tail -20 gpurun_out/ff_rates_c2_hub.log; exit 1; }
grep -v "ff=0" gpurun_out/ff_rates_c2_hub.log
