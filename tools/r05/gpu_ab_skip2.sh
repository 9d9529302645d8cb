#!/bin/bash
# round 5 A/B: the lane kernel's settle scan also skips the entries no (a read-off skip too: slower, dropped)
# lane of the wave needs (default build) against the relaxation skip alone (lib/variants/relaxonly):
# c4 at 1M and at 125k alternated, then the default
# build's lane-mode parity tests and the configs[3] lane-kernel oracle checks
set -o pipefail
mkdir -p gpurun_out
V=marshrutka_amd/lib/variants/relaxonly/libmarshrutka_pf.so
for i in 1 2; do
  for q in 1000000 125000; do
    MR_LIB_PATH=$V timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-reps 0 --queries $q > gpurun_out/ab_relax_${q}_$i.json 2> gpurun_out/ab_relax_${q}_$i.err || { tail -20 gpurun_out/ab_relax_${q}_$i.err; exit 1; }
    timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-reps 0 --queries $q > gpurun_out/ab_skip3_${q}_$i.json 2> gpurun_out/ab_skip3_${q}_$i.err || { tail -20 gpurun_out/ab_skip3_${q}_$i.err; exit 1; }
    python -c "
import json
for t in ('relax','skip3'):
    d=json.load(open('gpurun_out/ab_%s_${q}_$i.json'%t)); print(t, $q, round(d['value']/1e6,1), 'Mq/s kernel', round(d['roofline']['kernel_ms'],4))"
  done
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_full_scale.py \
  -k "lane or c4 or fleetfoot_hub or golden" > gpurun_out/ab_skip3_tests.log 2>&1 || { tail -40 gpurun_out/ab_skip3_tests.log; exit 1; }
tail -2 gpurun_out/ab_skip3_tests.log
