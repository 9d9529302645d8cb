#!/bin/bash
# lane-kernel build variants A/B on c4 (MR_LIB_PATH), then the shard fixture
set -o pipefail
mkdir -p gpurun_out/r06
for v in base w3 pf2 pf0 base; do
  if [ $v = base ]; then L=""; else L="marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so"; fi
  MR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/lane_ab_$v.log 2>&1 || { tail -20 gpurun_out/r06/lane_ab_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06/lane_ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_dev_group.py -k many_invalid -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/devgroup.log 2>&1 && tail -1 gpurun_out/r06/devgroup.log && timeout -k 10 300 python -u tests/golden/make_shard_records.py > gpurun_out/r06/make_shard.log 2>&1 && cp tests/golden/shard_records.npz gpurun_out/r06/shard_records.npz
