#!/bin/bash
# c3 fill-kernel experiments: grid size
set -e
for gx in 1024 2048 4096; do
    v=$(MR_FILL_GX=$gx timeout -k 10 120 python3 bench.py --workload c3 --steps 5 --warmup 1 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print(round(d['ms_per_step'],3))")
    echo "gx=$gx ms=$v"
done
