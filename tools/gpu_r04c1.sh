#!/bin/bash
# plan-create phases of the small batches (c1, c2)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04c1
mkdir -p $O
MR_TIMING=1 timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline --steps 20 --warmup 3 --e2e-reps 7 > $O/bench_c2.json 2> $O/bench_c2.err && echo c2-ok || exit 1
MR_TIMING=1 timeout -k 10 200 python bench.py --workload c1 --no-cpu-baseline --steps 20 --warmup 3 --e2e-reps 7 > $O/bench_c1.json 2> $O/bench_c1.err && echo c1-ok || exit 1
