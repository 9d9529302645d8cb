"""GPU probe (not product code): device build time of the grid's region table
(mr_grid_region_table, csrc/mr_k_region.hip) on the configs[3] and configs[4] maps.
usage: python tools/r06/region_time.py [c4|c5 ...]  (MR_REGION_SERIAL=1: the serial kernels)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap  # noqa: E402

for w in sys.argv[1:] or ["c4", "c5"]:
    if w == "c4":
        m = SyntheticMap(1025, campfires_per_homeland=4, seed=4096)
    else:
        with open(os.path.join(ROOT, "tests", "golden", "full_scale", "c5.json")) as f:
            m = SyntheticMap(**json.load(f)["map"])
    g = pf.MapGrid.from_array(m.cells_array())
    for h in range(4 if w == "c4" else 1):
        n, ms, _ = g.region_table(h, fetch=False)
        print(f"{w} homeland {h}: {n} regions, table build {ms:.2f} ms (wall, upload of the regions included)", flush=True)
    del g
