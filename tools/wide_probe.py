#!/usr/bin/env python3
"""Kernel time of the wide hub solver on c5-like maps under parameter variants
(SoE on/off isolates the region-row scan and the SoE relaxations; sort orders).

    python tools/wide_probe.py [--size 4097] [--queries 10000]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from marshrutka_amd import build, pathfinder  # noqa: E402
from marshrutka_amd.abi import SORT_LEGS, SORT_MONEY, SORT_TIME, Params  # noqa: E402
from marshrutka_amd.mapgen import SyntheticMap, random_queries  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=4097)
    ap.add_argument("--queries", type=int, default=10000)
    ap.add_argument("--k", type=int, default=64)
    a = ap.parse_args()
    build.build()
    m = SyntheticMap(a.size, campfires_per_homeland=a.k, seed=a.size, clustered=True)
    g = pathfinder.MapGrid.from_array(m.cells_array())
    qs = random_queries(m, a.queries, 45)
    variants = {
        "time_money": Params(sort_by=(SORT_TIME, SORT_MONEY)),
        "time_money_nosoe": Params(sort_by=(SORT_TIME, SORT_MONEY), use_soe=False),
        "money_legs": Params(sort_by=(SORT_MONEY, SORT_LEGS)),
        "legs_money": Params(),
        "legs_money_nocaravan": Params(use_caravans=False),
    }
    for name, p in variants.items():
        plan = pathfinder.Plan(g, p, qs)
        for _ in range(2):
            plan.run()
        plan.kernel_ms()
        for _ in range(5):
            plan.run()
        ms, n = plan.kernel_ms()
        st = plan.stats()
        print(json.dumps({"variant": name, "kernel_ms": round(ms, 3), "qps": round(a.queries / ms * 1e3),
                          "solver": st["solver"], "fallback": st["fallback_sources"],
                          "boundary_cells": st["region_boundary_cells"], "regions": st["num_regions"]}), flush=True)
        del plan


if __name__ == "__main__":
    main()
