#!/bin/bash
# wire fetch: the fetch parity tests, then the c4 end-to-end (pageable and page-locked)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_scale.py -k "fetch or wire or e2e or end_to_end or decode" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/fetch_tests.log 2>&1 || { tail -60 gpurun_out/r06/fetch_tests.log; exit 1; }
tail -3 gpurun_out/r06/fetch_tests.log
timeout -k 10 300 python -u bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r06/bench_c4_fetch.log 2>gpurun_out/r06/bench_c4_fetch.err || { tail -30 gpurun_out/r06/bench_c4_fetch.err; exit 1; }
python - <<'P'
import json
d = json.loads(open("gpurun_out/r06/bench_c4_fetch.log").read().strip().splitlines()[-1])
for k in ("end_to_end", "end_to_end_pinned"):
    print(k, {x: d[k][x] for x in ("e2e_queries_per_s", "ms", "plan_create_ms", "run_ms", "fetch_ms")})
P
