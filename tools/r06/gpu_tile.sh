#!/bin/bash
# round 6: the tile sweep — Time-first Fleetfoot probes (MR_CERT_DEBUG), a kernel trace,
# the certificate tests
set -o pipefail
mkdir -p gpurun_out/r06/prof
export TMPDIR=/tmp
for FF in 2 1; do
  MR_CERT_DEBUG=1 timeout -k 10 120 python -u tools/r05/ff_one.py $FF 1 2 3 > gpurun_out/r06/ff_one_$FF.log 2>&1 || { tail -30 gpurun_out/r06/ff_one_$FF.log; exit 1; }
  grep "slot 0 \|pass" gpurun_out/r06/ff_one_$FF.log
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof/ff2 -o run --output-format csv -- python3 tools/r05/ff_one.py 2 1 2 5 > gpurun_out/r06/prof/ff2.log 2>&1 || exit 1
grep -E "cert_|hub_|fill_kernel|solve" gpurun_out/r06/prof/ff2/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_cert.py \
  > gpurun_out/r06/tests_cert.log 2>&1 || { tail -60 gpurun_out/r06/tests_cert.log; exit 1; }
tail -2 gpurun_out/r06/tests_cert.log
