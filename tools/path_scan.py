"""Diagnostic: queries/s of each solver path across map sizes (10k uniform queries)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import SORT_LEGS, SORT_MONEY, SORT_TIME, Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

CASES = [("ff0 legs", Params()), ("ff1 legs", Params(fleetfoot=1)),
         ("ff0 time", Params(sort_by=(SORT_TIME, SORT_MONEY))), ("ff2 time", Params(fleetfoot=2, sort_by=(SORT_TIME, SORT_LEGS))),
         ("ff3 money", Params(fleetfoot=3, sort_by=(SORT_MONEY, SORT_LEGS)))]
for size in (65, 129, 255):
    m = SyntheticMap(size, campfires_per_homeland=4, seed=size)
    g = pathfinder.MapGrid(m.cells())
    qs = random_queries(m, 10000, 5)
    for name, p in CASES:
        plan = pathfinder.Plan(g, p, qs)
        plan.run()
        plan.kernel_ms()
        t0 = time.perf_counter()
        n = 3
        for _ in range(n):
            plan.run()
        ms, _ = plan.kernel_ms()
        st = plan.stats()
        print(f"S={size} {name:10s} solver={st['solver']:9s} fb={st['fallback_sources']:5d} "
              f"kernel_ms={ms:9.3f} q/s={10000 / (ms * 1e-3):12.0f}", flush=True)
