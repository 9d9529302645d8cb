#!/bin/bash
# world-1 RCCL path (wire gather) against the plain step, final build; then its kernel trace
set -o pipefail
mkdir -p gpurun_out/r06
for f in plain dist1 plain dist1; do
  if [ $f = dist1 ]; then E="MR_BENCH_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517"; else E=""; fi
  env $E timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/final_$f.log 2>&1 || { tail -20 gpurun_out/r06/final_$f.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/r06/final_$f.log').read().strip().splitlines()[-1])
print('$f', d['ms_per_step'], d['value'], d.get('gather_check'))"
done
bash tools/r06/gpu_prof_dist1.sh
