#!/bin/bash
# round 5 A/B (kept, no time change; the variant macro is gone since): the lane kernel's relaxation with its first two candidates combined into new
# registers (ltm_min) and a mask-only take (the default build) against the previous code
# (an MR_LANE_TAKE_COPY variant build): c4 bench lines alternated, then the default build's
# lane-mode parity tests and the configs[3] lane-kernel oracle checks
set -o pipefail
mkdir -p gpurun_out
V=marshrutka_amd/lib/variants/copy/libmarshrutka_pf.so
for i in 1 2; do
  MR_LIB_PATH=$V timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-reps 0 > gpurun_out/ab_copy_$i.json 2> gpurun_out/ab_copy_$i.err || { tail -20 gpurun_out/ab_copy_$i.err; exit 1; }
  timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-reps 0 > gpurun_out/ab_min_$i.json 2> gpurun_out/ab_min_$i.err || { tail -20 gpurun_out/ab_min_$i.err; exit 1; }
  python -c "
import json
for t in ('copy','min'):
    d=json.load(open('gpurun_out/ab_%s_$i.json'%t)); print(t, round(d['value']/1e6,1), 'Mq/s kernel', round(d['roofline']['kernel_ms'],4))"
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_full_scale.py \
  -k "lane or c4 or fleetfoot_hub or golden" > gpurun_out/ab_min_tests.log 2>&1 || { tail -40 gpurun_out/ab_min_tests.log; exit 1; }
tail -2 gpurun_out/ab_min_tests.log
