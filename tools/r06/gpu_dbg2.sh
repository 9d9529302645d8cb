#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
for FF in 2 3; do
MR_CERT_DEBUG=1 timeout -k 10 200 python -u tools/probes/cert_dbg.py $FF > gpurun_out/r06/certdbg_$FF.log 2>&1 || { tail -20 gpurun_out/r06/certdbg_$FF.log; exit 1; }
grep "handed" gpurun_out/r06/certdbg_$FF.log
grep "slot" gpurun_out/r06/certdbg_$FF.log | grep -v "fails 0" | cut -c1-220 | head -20
done
