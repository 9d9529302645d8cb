#!/bin/bash
# round 4: lane kernel read-off ties among the tied boundaries only: parity, c4 bench x2
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t_parity_r04ze.log 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > gpurun_out/b_c4_mc$i.json 2> gpurun_out/b_c4_mc$i.err || exit 1
done
