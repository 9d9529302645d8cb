"""Diagnostic: one source, repeated runs (latency of a single hub solve)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)
g = pathfinder.MapGrid(m.cells())
q = random_queries(m, 1, 5)
plan = pathfinder.Plan(g, Params(), q)
for _ in range(20):
    plan.run()
ms, n = plan.kernel_ms()
print(f"1 source: {ms:.4f} ms per run over {n}", flush=True)
pathfinder.lib().mr_plan_destroy(plan.handle)
plan.handle = None
