"""GPU probe: the sources the non-linear hub hands to the SSSP fallback (Time-first,
Fleetfoot 1..3, the ff_rates.py batch), with their destinations in the batch, as JSON
for the CPU-side certificate experiments.  Not product code."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402


def main(size=1025, nq=125000, out="gpurun_out/ff_dump.json"):
    m = SyntheticMap(size, campfires_per_homeland=4, seed=2024)
    g = pf.MapGrid(m.cells())
    qs = random_queries(m, nq, 7)
    res = []
    for ff in (1, 2, 3):
        for s in ((1, 0), (1, 2)):
            plan = pf.Plan(g, Params(fleetfoot=ff, sort_by=s), qs)
            plan.run()
            fb = plan.fallback_sources()
            keys = {tuple(c.to_tuple()) if hasattr(c, "to_tuple") else repr(c) for c in fb}
            dsts = {}
            for a, b in qs:
                for c in fb:
                    if a == c:
                        dsts.setdefault(repr(c), []).append(repr(b))
            res.append({"ff": ff, "sort_by": s, "fallback": [repr(c) for c in fb], "dsts": dsts,
                        "n_keys": len(keys)})
            print(ff, s, len(fb), flush=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
