"""GPU probe: the non-linear hub (Fleetfoot 1..3) on c2/c4-like batches — share of
sources it certifies, and pass time, per comparator order.  Not product code."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402

SORTS = [(0, 2), (0, 1), (2, 0), (2, 1), (1, 0), (1, 2)]  # Legs=0 Time=1 Money=2


def main(size=65, nq=10000, steps=5, seed=2024):
    m = SyntheticMap(size, campfires_per_homeland=4, seed=seed)
    g = pf.MapGrid(m.cells())
    qs = random_queries(m, nq, 7)
    for ff in (0, 1, 2, 3):
        for s in SORTS:
            plan = pf.Plan(g, Params(fleetfoot=ff, sort_by=s), qs)
            plan.run()
            plan.kernel_ms()  # (drops the first pass: a kernel's first launch loads its code object)
            t = time.time()
            for _ in range(steps):
                plan.run()
            plan.fetch_raw()
            wall = (time.time() - t) / steps
            st = plan.stats()
            ms, n = plan.kernel_ms()
            print(f"S={size} seed={seed} ff={ff} sort={s}: solver {st['solver']} fallback {st['fallback_sources']}/"
                  f"{st['num_sources']} kernel {ms:.3f} ms  {nq / (ms * 1e-3) / 1e6:.2f} M q/s (wall {wall * 1e3:.2f} ms)",
                  flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
