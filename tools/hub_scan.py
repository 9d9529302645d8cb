"""Diagnostic: solve-kernel time vs number of sources (latency vs throughput)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

for size, seed in ((65, 2024), (1025, 4096)):
    m = SyntheticMap(size, campfires_per_homeland=4, seed=seed)
    g = pathfinder.MapGrid(m.cells())
    allq = random_queries(m, 200000 if size > 100 else 10000, seed + 17)
    for k in (1, 64, 1024, 4096, 16384, 65536, 131072):
        seen, qs = set(), []
        for a, b in allq:
            if a not in seen:
                if len(seen) == k:
                    continue
                seen.add(a)
            qs.append((a, b))
        if len(seen) < k:
            break
        plan = pathfinder.Plan(g, Params(), qs)
        for _ in range(3):
            plan.run()
        plan.kernel_ms()
        for _ in range(5):
            plan.run()
        ms, _ = plan.kernel_ms()
        st = plan.stats()
        print(f"S={size} sources={plan.num_sources} queries={len(qs)} kernel_ms={ms:.4f} "
              f"per_source_us={ms * 1e3 / plan.num_sources:.3f} hub_wg={st['hub_workgroups']} "
              f"fallback={st['fallback_sources']}", flush=True)
