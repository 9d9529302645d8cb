#!/bin/bash
# Round 4 host path: fetch / plan parity tests, then 125k and 1M end to end with phase timings
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "fetch or capacity or invalid or plan or c4 or e2e or find_path or full_scale" > $O/gpu_tests.log 2>&1 && echo tests-ok || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
MR_TIMING=1 timeout -k 10 200 python bench.py --queries 125000 --steps 10 --warmup 2 --no-cpu-baseline --e2e-reps 7 > $O/bench_125k.json 2> $O/bench_125k.err && echo 125k-ok || exit 1
MR_TIMING=1 timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --e2e-reps 5 > $O/bench_1m.json 2> $O/bench_1m.err && echo 1m-ok || exit 1
