#!/bin/bash
# round 5: device grouping of query batches — equality with the host grouping, the
# configs[3] parity tests on the new default path, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_dev_group.py tests/test_gpu_full_scale.py -k "dev_group or grouping or c4" \
  > gpurun_out/tests_devgroup.log 2>&1 || { tail -80 gpurun_out/tests_devgroup.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/tests_devgroup.log | tail -20
MR_TIMING=1 timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_devgroup.json 2> gpurun_out/bench_devgroup.err || { tail -30 gpurun_out/bench_devgroup.err; exit 1; }
grep MR_TIMING gpurun_out/bench_devgroup.err | tail -8
python -c "import json; d=json.load(open('gpurun_out/bench_devgroup.json')); print(d['value'], d['end_to_end'], d['end_to_end_pinned'])"
MR_TIMING=1 timeout -k 10 300 python bench.py --queries 125000 --no-cpu-baseline > gpurun_out/bench_devgroup_125k.json 2> gpurun_out/bench_devgroup_125k.err || { tail -30 gpurun_out/bench_devgroup_125k.err; exit 1; }
grep MR_TIMING gpurun_out/bench_devgroup_125k.err | tail -4
python -c "import json; d=json.load(open('gpurun_out/bench_devgroup_125k.json')); print(d['value'], d['end_to_end'], d['end_to_end_pinned'])"
