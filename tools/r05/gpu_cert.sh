#!/bin/bash
# round 5: the queued repair sweep — certificate tests, the parity suite's fallback
# modes, then kernel traces of the Fleetfoot 2 / 1 Time-first fallback and the rates
set -o pipefail
mkdir -p gpurun_out/certprof
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_cert.py tests/test_gpu_parity.py -k "cert or fallback or Fleetfoot or fleetfoot or staging" \
  > gpurun_out/tests_cert.log 2>&1 || { tail -80 gpurun_out/tests_cert.log; exit 1; }
grep -E "passed|failed" gpurun_out/tests_cert.log | tail -3
for FF in 2 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/certprof/ff$FF -o run --output-format csv -- python3 tools/r05/ff_one.py $FF 1 2 5 > gpurun_out/certprof/ff$FF.log 2>&1 || exit 1
  grep "pass" gpurun_out/certprof/ff$FF.log
  grep -E "sweep|hub_kernel|hub_lane|cert_|fill_kernel" gpurun_out/certprof/ff$FF/run_kernel_stats.csv | cut -d, -f1-4
done
timeout -k 10 400 python tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_q.log 2>&1 || exit 1
grep "sort=(1" gpurun_out/ff_rates_q.log
