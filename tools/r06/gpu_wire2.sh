#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "wire or fetch" -x -q --timeout 200 --timeout-method thread > gpurun_out/r06/wire_tests.log 2>&1 || { tail -40 gpurun_out/r06/wire_tests.log; exit 1; }
tail -1 gpurun_out/r06/wire_tests.log
bash tools/r06/gpu_prof_dist1.sh || exit 1
python3 - <<'P'
import csv
for r in list(csv.DictReader(open("gpurun_out/r06/dist1_kernel_stats.csv")))[:6]:
    print(r["Name"][:40], r["Calls"], r["AverageNs"])
P
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/bench_c4_plain.log 2>&1 || exit 1
MR_BENCH_DIST=1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29514 timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/bench_c4_dist1.log 2>&1 || exit 1
python3 - <<'P'
import json
for f in ("plain", "dist1"):
    d = json.loads(open(f"gpurun_out/r06/bench_c4_{f}.log").read().strip().splitlines()[-1])
    print(f, d["ms_per_step"], d["value"], d.get("gather_check"))
P
