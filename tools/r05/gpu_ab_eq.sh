#!/bin/bash
# round 5 A/B (not kept, DESIGN.md §3a‴): the lane kernel's offer with one borrow chain and equality masks (an MR_LANE_EQ
# variant build) against the default build: c4 bench lines alternated, then the variant's
# lane-mode parity tests and its configs[3] lane-kernel oracle check
set -o pipefail
mkdir -p gpurun_out
V=marshrutka_amd/lib/variants/eq/libmarshrutka_pf.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-reps 0 > gpurun_out/ab_base_$i.json 2> gpurun_out/ab_base_$i.err || { tail -20 gpurun_out/ab_base_$i.err; exit 1; }
  MR_LIB_PATH=$V timeout -k 10 300 python bench.py --no-cpu-baseline --e2e-reps 0 > gpurun_out/ab_eq_$i.json 2> gpurun_out/ab_eq_$i.err || { tail -20 gpurun_out/ab_eq_$i.err; exit 1; }
  python -c "
import json
for t in ('base','eq'):
    d=json.load(open('gpurun_out/ab_%s_$i.json'%t)); print(t, round(d['value']/1e6,1), 'Mq/s kernel', round(d['roofline']['kernel_ms'],4), 'parity', d.get('parity'))"
done
MR_LIB_PATH=$V timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_full_scale.py \
  -k "lane or c4_lane or overflow or fleetfoot_hub" > gpurun_out/ab_eq_tests.log 2>&1 || { tail -40 gpurun_out/ab_eq_tests.log; exit 1; }
tail -2 gpurun_out/ab_eq_tests.log
