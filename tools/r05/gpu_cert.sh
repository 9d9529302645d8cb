#!/bin/bash
# round 5: the dirty-queue repair sweep — certificate tests, the parity suite's fallback
# modes, then the Fleetfoot rates (queued sweep, and the full sweep for A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_cert.py tests/test_gpu_parity.py -k "cert or fallback or Fleetfoot or fleetfoot" \
  > gpurun_out/tests_cert.log 2>&1 || { tail -80 gpurun_out/tests_cert.log; exit 1; }
grep -E "passed|failed" gpurun_out/tests_cert.log | tail -3
timeout -k 10 400 python tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_q.log 2>&1 || exit 1
grep "sort=(1" gpurun_out/ff_rates_q.log
MR_DBG_FLAGS=256 timeout -k 10 400 python tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_full.log 2>&1 || exit 1
grep "sort=(1" gpurun_out/ff_rates_full.log
