#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
for FF in 2 1; do
  MR_CERT_DEBUG=1 timeout -k 10 120 python -u tools/r05/ff_one.py $FF 1 2 2 > gpurun_out/r06/ff_one_$FF.log 2>&1 || { tail -30 gpurun_out/r06/ff_one_$FF.log; exit 1; }
  grep "pass" gpurun_out/r06/ff_one_$FF.log
done
