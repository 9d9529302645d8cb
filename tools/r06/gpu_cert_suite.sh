#!/bin/bash
# round 6: the tile sweep under the certificate-related GPU tests (parity suite fallback
# modes, full-scale Fleetfoot tests), then c4's own map (seed 4096) Time-first Fleetfoot 1-3
set -o pipefail
mkdir -p gpurun_out/r06
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_cert.py tests/test_gpu_parity.py tests/test_gpu_full_scale.py -k "cert or fallback or Fleetfoot or fleetfoot or staging" \
  > gpurun_out/r06/tests_cert_suite.log 2>&1 || { tail -80 gpurun_out/r06/tests_cert_suite.log; exit 1; }
grep -E "passed|failed" gpurun_out/r06/tests_cert_suite.log | tail -3
timeout -k 10 400 python -u tools/r06/ff_c4map.py > gpurun_out/r06/ff_c4map.log 2>&1 || { tail -20 gpurun_out/r06/ff_c4map.log; exit 1; }
cat gpurun_out/r06/ff_c4map.log
