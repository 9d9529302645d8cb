#!/bin/bash
# round 5: c2 on the group kernel at 16 against 32 lanes a source (MR_HUB_GROUP), alternated
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  for g in 16 32; do
    MR_HUB_GROUP=$g timeout -k 10 300 python bench.py --workload c2 --no-cpu-baseline --e2e-reps 0 > gpurun_out/c2_g${g}_$i.json 2> gpurun_out/c2_g${g}_$i.err || { tail -20 gpurun_out/c2_g${g}_$i.err; exit 1; }
    python -c "
import json
d=json.load(open('gpurun_out/c2_g${g}_$i.json')); print('G=$g', round(d['value']/1e6,1), 'Mq/s kernel', round(d['roofline']['kernel_ms'],4), d['roofline']['kernel'])"
  done
done
