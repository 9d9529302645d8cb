#!/bin/bash
# per certificate slot: the first check's failing box (MR_CERT_NOSWEEP) and the last
# check's after the sweep, Time-first Fleetfoot 2 / 3 on c4's map
set -o pipefail
mkdir -p gpurun_out
for FF in 2 3; do
  MR_CERT_NOSWEEP=1 timeout -k 10 200 python -u tools/probes/cert_dbg.py $FF > gpurun_out/certdbg_first_$FF.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/probes/cert_dbg.py $FF > gpurun_out/certdbg_last_$FF.log 2>&1 || exit 1
done
for f in gpurun_out/certdbg_*.log; do echo == $f; grep -E "ff|MR_CERT_DEBUG" $f | head -14; done
