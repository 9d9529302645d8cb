"""c4-size fetch timing: mr_plan_fetch through the wire rows vs the device decoder
(MR_TIMING=1 breakdown on stderr), into reused caller arrays."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
m = SyntheticMap(1025, campfires_per_homeland=4, seed=4096)
grid = pathfinder.MapGrid.from_array(m.cells_array())
V = m.size * m.size
rng = np.random.default_rng(7)
qa = m.query_array(rng.integers(0, V, n), rng.integers(0, V, n))
bufs = pathfinder.fetch_buffers(n, 4)
for b in bufs:
    np.frombuffer(b, dtype=np.uint8).fill(0)
plan = pathfinder.Plan(grid, Params(), None, max_cmds=4, query_array=qa)
plan.run()
plan.wait()
fresh = os.environ.get("FRESH") == "1"
for mode, pin in (("1", 0), ("0", 0), ("1", 1), ("0", 1), ("1", 0)):
    os.environ["MR_FETCH_WIRE"] = mode
    if pin:
        for b in bufs:
            pathfinder.pin_host(b)
    ts = []
    for _ in range(4):
        if fresh:  # a new plan per fetch (bench.py's end_to_end)
            del plan
            plan = pathfinder.Plan(grid, Params(), None, max_cmds=4, query_array=qa)
            plan.run()
            plan.wait()
        t0 = time.perf_counter()
        plan.fetch_raw(bufs)
        ts.append((time.perf_counter() - t0) * 1e3)
    if pin:
        for b in bufs:
            pathfinder.unpin_host(b)
    print(f"MR_FETCH_WIRE={mode} pinned={pin}: fetch ms {[round(t, 2) for t in ts]}", flush=True)
