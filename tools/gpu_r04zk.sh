#!/bin/bash
# round 4: end-to-end phases of the 1M batch (MR_TIMING)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04zk
mkdir -p $O
MR_TIMING=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-reps 5 > $O/b_c4.json 2> $O/b_c4.err
