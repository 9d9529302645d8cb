#!/bin/bash
set -o pipefail
bash tools/r06/gpu_suite.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r06/bench_c4_final4.json 2> gpurun_out/r06/bench_c4_final4.err || { tail -20 gpurun_out/r06/bench_c4_final4.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r06/bench_c4_final4.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'])
for k in ('end_to_end','end_to_end_pinned'): print(k, {x: round(d[k][x],3) for x in ('e2e_queries_per_s','ms','plan_create_ms','run_ms','fetch_ms')})"
