#!/bin/bash
# fetch path tests, the default bench line (driver's command), then c3 and c5 profiles
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fetch or wire" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06/fetch_tests2.log 2>&1 || { tail -30 gpurun_out/r06/fetch_tests2.log; exit 1; }
tail -1 gpurun_out/r06/fetch_tests2.log
timeout -k 10 300 python bench.py > gpurun_out/r06/bench_c4_final.json 2> gpurun_out/r06/bench_c4_final.err || { tail -20 gpurun_out/r06/bench_c4_final.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r06/bench_c4_final.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['parity'])
for k in ('end_to_end','end_to_end_pinned'): print(k, {x: round(d[k][x],3) for x in ('e2e_queries_per_s','ms','plan_create_ms','run_ms','fetch_ms')})"
bash tools/profile_round.sh r06 "c3 c5"
