#!/bin/bash
# the full-scale Fleetfoot tests, the certificate tests, then one Time-first Fleetfoot 1
# batch on c4's map (tens of handed-over sources) with the default slots and with 8
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_full_scale.py tests/test_gpu_cert.py -x -v --timeout 600 --timeout-method thread -k "fleetfoot or cert" > gpurun_out/tests_ff_full.log 2>&1 || { tail -n 30 gpurun_out/tests_ff_full.log; exit 1; }
tail -n 3 gpurun_out/tests_ff_full.log
cat > /tmp/ff_c4map.py <<'PY'
import os, sys
sys.path.insert(0, os.getcwd())
from marshrutka_amd import pathfinder as pf
from marshrutka_amd.abi import Params
from marshrutka_amd.mapgen import SyntheticMap, random_query_cells
m = SyntheticMap(1025, campfires_per_homeland=4, seed=4096)
arr = m.cells_array()
g = pf.MapGrid.from_array(arr)
src, dst = random_query_cells(m, 125000, 5001)
for ff in (1, 2, 3):
    plan = pf.Plan(g, Params(fleetfoot=ff, sort_by=(1, 0)), None, max_cmds=8, query_array=m.query_array(src, dst, arr))
    plan.run(); plan.kernel_ms()
    for _ in range(3): plan.run()
    ms, _ = plan.kernel_ms(); st = plan.stats()
    print(f"c4 map ff={ff} Time-first: fallback {st['fallback_sources']} certified {st['certified_sources']} pass {ms:.2f} ms  {125000 / ms / 1e3:.1f} M q/s", flush=True)
PY
timeout -k 10 300 python -u /tmp/ff_c4map.py || exit 1
MR_CERT_SLOTS=8 timeout -k 10 300 python -u /tmp/ff_c4map.py || exit 1
