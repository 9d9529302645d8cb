#!/bin/bash
# the N > 1 bench path rehearsed with two gloo ranks on one GPU (host-staged wire gather)
set -o pipefail
mkdir -p gpurun_out/r06
MR_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/gloo2_c4.json 2> gpurun_out/r06/gloo2_c4.err || { tail -30 gpurun_out/r06/gloo2_c4.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r06/gloo2_c4.json').read().strip().splitlines()[-1])
print(d['n_gpus'], d['value'], d['ms_per_step'], d.get('gather_check'), d['config'].get('parallelism'))"
