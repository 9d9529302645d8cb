"""Diagnostic: SSSP path with many specials (c5-like) at growing S."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import SORT_LEGS, SORT_MONEY, SORT_TIME, Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

for size in (129, 257, 513):
    m = SyntheticMap(size, campfires_per_homeland=64, seed=size, clustered=True)
    g = pathfinder.MapGrid(m.cells())
    qs = random_queries(m, 1000, 5)
    for name, p in (("time", Params(sort_by=(SORT_TIME, SORT_LEGS))), ("money", Params(sort_by=(SORT_MONEY, SORT_TIME)))):
        plan = pathfinder.Plan(g, p, qs)
        plan.run()
        ms, _ = plan.kernel_ms()
        st = plan.stats()
        print(f"S={size} NS={st['num_specials']} {name} solver={st['solver']} state_lds={st['grid_state_in_lds']} "
              f"kernel_ms={ms:.2f} q/s={1000 / (ms * 1e-3):.0f}", flush=True)
