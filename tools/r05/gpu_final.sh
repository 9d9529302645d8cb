#!/bin/bash
# round 5, final tree: the default bench line (its issue figures from the committed SQ
# summary), then the whole GPU suite and smoke
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_c4_final.json 2> gpurun_out/bench_c4_final.err || { tail -20 gpurun_out/bench_c4_final.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c4_final.json')); print(d['value'], d['roofline']['kernel_ms'], d['parity'])"
bash tools/r05/gpu_suite.sh
