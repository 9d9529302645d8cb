#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 400 python -u tools/r06/ff_c4map.py > gpurun_out/r06/ff_c4map.log 2>&1 || { tail -20 gpurun_out/r06/ff_c4map.log; exit 1; }
cat gpurun_out/r06/ff_c4map.log
for FF in 2 1; do
  timeout -k 10 120 python -u tools/r05/ff_one.py $FF 1 2 3 || exit 1
done
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_cert.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -k "cert or fallback or Fleetfoot or fleetfoot or staging" \
  > gpurun_out/r06/tests_cert_suite.log 2>&1 || { tail -80 gpurun_out/r06/tests_cert_suite.log; exit 1; }
tail -2 gpurun_out/r06/tests_cert_suite.log
