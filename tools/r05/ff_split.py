"""GPU probe: where the non-linear hub's pass time goes — certification of destinations
on/off (MR_DBG_FLAGS=8 skips it: labels unchecked, timing only) and the linear hub_kernel
at the same batch.  Not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from marshrutka_amd import pathfinder as pf  # noqa: E402
from marshrutka_amd.abi import Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402


def t(g, qs, params, env, steps=5):
    for k, v in env.items():
        os.environ[k] = v
    plan = pf.Plan(g, params, qs)
    for k in env:
        del os.environ[k]
    plan.run()
    for _ in range(steps):
        plan.run()
    ms, n = plan.kernel_ms()
    return ms, plan.stats()["solver"], plan.stats()["fallback_sources"]


def main(size=1025, nq=125000):
    m = SyntheticMap(size, campfires_per_homeland=4, seed=2024)
    g = pf.MapGrid(m.cells())
    qs = random_queries(m, nq, 7)
    for s in [(0, 2), (2, 0), (1, 0)]:
        print(f"ff=0 sort={s} hub_kernel {t(g, qs, Params(sort_by=s), {'MR_HUB_LANE': '0', 'MR_HUB_GROUP': '0'})}",
              flush=True)
        for ff in (1, 3):
            p = Params(fleetfoot=ff, sort_by=s)
            print(f"ff={ff} sort={s} full {t(g, qs, p, {})} nocert {t(g, qs, p, {'MR_DBG_FLAGS': '8'})}", flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
