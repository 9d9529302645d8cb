#!/bin/bash
# Fleetfoot rates on the c4-size (1025^2, 125k) and c2-size (65^2, 10k) batches; the c2
# batch also with Fleetfoot kept on hub_kernel (MR_LANE_NONLIN=0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ff_rates.py 1025 125000 5 > gpurun_out/ff_rates_c4.log 2>&1 || { tail -20 gpurun_out/ff_rates_c4.log; exit 1; }
timeout -k 10 300 python -u tools/ff_rates.py 65 10000 5 > gpurun_out/ff_rates_c2.log 2>&1 || { tail -20 gpurun_out/ff_rates_c2.log; exit 1; }
MR_LANE_NONLIN=0 timeout -k 10 300 python -u tools/ff_rates.py 65 10000 5 > gpurun_out/ff_rates_c2_hub.log 2>&1 || { tail -20 gpurun_out/ff_rates_c2_hub.log; exit 1; }
cat gpurun_out/ff_rates_c4.log; echo; cat gpurun_out/ff_rates_c2.log; echo; grep -v "ff=0" gpurun_out/ff_rates_c2_hub.log
