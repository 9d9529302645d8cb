#!/bin/bash
# round 6, first GPU call: the parallel region table and the tile sweep (certificate tests,
# Time-first Fleetfoot probes with MR_CERT_DEBUG, A/B against the round-5 sweep)
set -o pipefail
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_region_table.py \
  > gpurun_out/r06/tests_region.log 2>&1 || { tail -40 gpurun_out/r06/tests_region.log; exit 1; }
tail -2 gpurun_out/r06/tests_region.log
timeout -k 10 200 python -u tools/r06/region_time.py c4 c5 > gpurun_out/r06/region_time.log 2>&1 || { tail -20 gpurun_out/r06/region_time.log; exit 1; }
MR_REGION_SERIAL=1 timeout -k 10 200 python -u tools/r06/region_time.py c4 c5 > gpurun_out/r06/region_time_serial.log 2>&1 || exit 1
cat gpurun_out/r06/region_time.log gpurun_out/r06/region_time_serial.log
for FF in 2 1; do
  MR_CERT_DEBUG=1 timeout -k 10 120 python -u tools/r05/ff_one.py $FF 1 2 3 > gpurun_out/r06/ff_one_$FF.log 2>&1 || { tail -30 gpurun_out/r06/ff_one_$FF.log; exit 1; }
  grep -v "fails 0" gpurun_out/r06/ff_one_$FF.log | tail -5
  MR_CERT_TILE=0 timeout -k 10 120 python -u tools/r05/ff_one.py $FF 1 2 3 > gpurun_out/r06/ff_one_${FF}_old.log 2>&1 || exit 1
  tail -1 gpurun_out/r06/ff_one_${FF}_old.log
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_cert.py \
  > gpurun_out/r06/tests_cert.log 2>&1 || { tail -60 gpurun_out/r06/tests_cert.log; exit 1; }
tail -2 gpurun_out/r06/tests_cert.log
