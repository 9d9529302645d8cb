#!/bin/bash
# after the prefetch default change: the lane-kernel parity tests, full-scale c4, bench, smoke
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_scale.py tests/test_gpu_dev_group.py -k "lane or c4 or fleetfoot or dev_group or device_grouping or golden or fetch or wire" -x -q --timeout 400 --timeout-method thread > gpurun_out/r06/final_c_tests.log 2>&1 || { tail -30 gpurun_out/r06/final_c_tests.log; exit 1; }
tail -1 gpurun_out/r06/final_c_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r06/bench_c4_final3.json 2> gpurun_out/r06/bench_c4_final3.err || { tail -20 gpurun_out/r06/bench_c4_final3.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r06/bench_c4_final3.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'])
for k in ('end_to_end','end_to_end_pinned'): print(k, {x: round(d[k][x],3) for x in ('e2e_queries_per_s','ms','plan_create_ms','run_ms','fetch_ms')})"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke3.log 2>&1 || { tail -20 gpurun_out/r06/smoke3.log; exit 1; }
tail -1 gpurun_out/r06/smoke3.log
