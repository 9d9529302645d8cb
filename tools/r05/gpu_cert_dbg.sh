#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for F in 0 256 512 768; do
echo "== flags $F"
MR_DBG_FLAGS=$F MR_CERT_DEBUG=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_cert.py -k flagged > gpurun_out/cert_dbg_$F.log 2>&1
grep -E "passed|failed" gpurun_out/cert_dbg_$F.log | tail -2
done
