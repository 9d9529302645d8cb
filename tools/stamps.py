"""Diagnostic: per-phase cycle breakdown of the solve kernel.

    python -m marshrutka_amd.build --diag
    MR_LIB_PATH=marshrutka_amd/lib/diag/libmarshrutka_pf.so python tools/stamps.py [c2|c4] [queries]

Prints the MR_STAMPS line of the diagnostic build (cycles summed over
workgroups, thread 0's view).  Diagnostic builds are never benchmarked.
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "c2"
nq = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
size = 65 if wl == "c2" else 1025
m = SyntheticMap(size, campfires_per_homeland=4, seed=2024 if wl == "c2" else 4096)
g = pathfinder.MapGrid(m.cells())
qs = random_queries(m, nq, 7)
plan = pathfinder.Plan(g, Params(), qs)
plan.run()
plan.kernel_ms()
t0 = time.perf_counter()
plan.run()
ms, _ = plan.kernel_ms()
print(f"{wl}: {nq} queries, {plan.num_sources} sources, kernel {ms:.3f} ms", flush=True)
pathfinder.lib().mr_plan_destroy(plan.handle)
plan.handle = None
