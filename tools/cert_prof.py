"""GPU probe: passes of the Time-first Fleetfoot plan on the ff_rates batch (1025^2,
125k queries), for a kernel trace of the certified fallback's launches.  Not product
code.  usage: python tools/cert_prof.py [ff] [passes]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402


def main(ff=2, passes=5):
    m = SyntheticMap(1025, campfires_per_homeland=4, seed=2024)
    g = pf.MapGrid(m.cells())
    qs = random_queries(m, 125000, 7)
    plan = pf.Plan(g, Params(fleetfoot=ff, sort_by=(1, 0)), qs)
    for _ in range(passes):
        plan.run()
    plan.fetch_raw()
    ms, n = plan.kernel_ms()
    print(plan.stats(), f"pass {ms:.3f} ms over {n}", flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
