"""GPU probe (not product code): Time-first Fleetfoot 1-3 on the c2-sized batch (65^2, 10k
queries): handed-over and certified sources and the pass time (run it under rocprofv3 for
the certificate kernels' split)."""
import os, sys
sys.path.insert(0, os.getcwd())
from marshrutka_amd import pathfinder as pf
from marshrutka_amd.abi import Params
from marshrutka_amd.mapgen import SyntheticMap, random_queries
m = SyntheticMap(65, campfires_per_homeland=4, seed=2024)
g = pf.MapGrid(m.cells())
qs = random_queries(m, 10000, 7)
for ff in (1, 2, 3):
    plan = pf.Plan(g, Params(fleetfoot=ff, sort_by=(1, 0)), qs)
    plan.run(); plan.kernel_ms()
    for _ in range(5): plan.run()
    ms, _ = plan.kernel_ms(); st = plan.stats()
    print(f"ff={ff}: fallback {st['fallback_sources']} certified {st['certified_sources']} pass {ms:.3f} ms", flush=True)
