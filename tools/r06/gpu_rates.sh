#!/bin/bash
# Fleetfoot rates at 1025^2 / 125k on seeds 2024 and 4096 (every order), c4-map hand-overs
set -o pipefail
mkdir -p gpurun_out/r06
for s in 2024 4096; do
  timeout -k 10 400 python -u tools/ff_rates.py 1025 125000 3 $s > gpurun_out/r06/ff_rates_$s.log 2>&1 || { tail -20 gpurun_out/r06/ff_rates_$s.log; exit 1; }
  grep "sort=(1" gpurun_out/r06/ff_rates_$s.log
done
timeout -k 10 300 python -u tools/r06/ff_c4map.py 4096 > gpurun_out/r06/ff_c4map.log 2>&1 || { tail -20 gpurun_out/r06/ff_c4map.log; exit 1; }
cat gpurun_out/r06/ff_c4map.log
