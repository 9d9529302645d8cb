#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
MR_CERT_DEBUG=1 timeout -k 10 200 python -u tools/probes/cert_dbg.py 1 > gpurun_out/r06/certdbg_1.log 2>&1 || { tail -20 gpurun_out/r06/certdbg_1.log; exit 1; }
grep "handed" gpurun_out/r06/certdbg_1.log
timeout -k 10 400 python -u tools/r06/ff_c4map.py > gpurun_out/r06/ff_c4map.log 2>&1 || { tail -20 gpurun_out/r06/ff_c4map.log; exit 1; }
cat gpurun_out/r06/ff_c4map.log
timeout -k 10 400 python -u tools/r06/ff_c4map.py 2024 > gpurun_out/r06/ff_2024map.log 2>&1 || { tail -20 gpurun_out/r06/ff_2024map.log; exit 1; }
cat gpurun_out/r06/ff_2024map.log
