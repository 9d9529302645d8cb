#!/bin/bash
# the whole GPU suite (one process), then smoke
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06/gpu_suite.log 2>&1 || { tail -60 gpurun_out/r06/gpu_suite.log; exit 1; }
tail -3 gpurun_out/r06/gpu_suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke.log 2>&1 || { tail -20 gpurun_out/r06/smoke.log; exit 1; }
tail -3 gpurun_out/r06/smoke.log
# (optional second stage: the c2-size Fleetfoot rates)
if [ "${RATES:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/ff_rates.py 65 10000 5 > gpurun_out/ff_rates_c2.log 2>&1 || { tail -20 gpurun_out/ff_rates_c2.log; exit 1; }
  grep "sort=(1" gpurun_out/ff_rates_c2.log
fi
