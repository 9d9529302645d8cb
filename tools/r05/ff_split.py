"""GPU probe: where the non-linear lane kernel's pass time goes — the settled specials'
certification (MR_DBG_FLAGS=4 skips it), the destinations' (=8), both (=12); labels
unchecked, timing only.  Not product code."""
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
    st = plan.stats()
    return f"{ms:.3f} ms (lane {st['lane_sources']}, fb {st['fallback_sources']})"


def main(size=1025, nq=125000):
    m = SyntheticMap(size, campfires_per_homeland=4, seed=2024)
    g = pf.MapGrid(m.cells())
    qs = random_queries(m, nq, 7)
    for s, ff in [((0, 2), 1), ((0, 2), 2), ((2, 0), 1), ((1, 0), 3), ((1, 0), 1)]:
        p = Params(fleetfoot=ff, sort_by=s)
        row = [f"ff={ff} sort={s}"]
        for dbg in ("0", "4", "8", "12"):
            row.append(f"dbg{dbg} {t(g, qs, p, {'MR_LANE_NONLIN': '1', 'MR_DBG_FLAGS': dbg})}")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
