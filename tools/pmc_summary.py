#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes into profiles/pmc_<workload>.json (bench.py's
roofline "traffic").

    python tools/pmc_summary.py --workload c2 --queries 10000 \\
        --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --out profiles/pmc_c2.json

Each pass is a separate `rocprofv3 --pmc <COUNTER> --kernel-trace --stats` run
of the same bench command (FETCH_SIZE and WRITE_SIZE do not fit one pass on
gfx950).  Per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are
kilobytes at the L2's fabric side; on gfx950 FETCH_SIZE reports half the bytes
of wide coalesced reads, so it is doubled; WRITE_SIZE is taken as is.  One
"launch" = one mr_plan_run (hub kernel + SSSP fallback kernel, or the SSSP
kernel alone; the fill's two launches), so the per-dispatch means of every solve
kernel instantiation are summed.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SOLVE_KERNELS = ("hub_group_kernel", "hub_lane_kernel", "hub_wide_kernel", "hub_fill_kernel", "hub_kernel", "solve_kernel", "fill_kernel")


def per_dispatch(path: str, counter: str):
    files = glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {path}")
    vals = defaultdict(list)
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                fam = next((k for k in SOLVE_KERNELS if k in name), None)
                if fam:  # per instantiation: a pass may launch two (the fill's wide-metric launch)
                    vals[(fam, name)].append(float(row["Counter_Value"]))
    per = defaultdict(lambda: [0.0, 0])
    for (fam, _), v in vals.items():
        per[fam][0] += sum(v) / len(v)
        per[fam][1] = max(per[fam][1], len(v))
    return {k: (v[0], v[1]) for k, v in per.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--queries", type=int, required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--kernels", default="", help="comma-separated kernels the roofline prices (default: all solve kernels)")
    a = ap.parse_args()
    keep = set(a.kernels.split(",")) if a.kernels else set(SOLVE_KERNELS)
    fe = {k: v for k, v in per_dispatch(a.fetch, "FETCH_SIZE").items() if k in keep}
    wr = {k: v for k, v in per_dispatch(a.write, "WRITE_SIZE").items() if k in keep}
    read_b = sum(2.0 * kb * 1024.0 for kb, _ in fe.values())   # gfx950: FETCH_SIZE = 1/2 of the bytes
    write_b = sum(kb * 1024.0 for kb, _ in wr.values())
    out = {
        "workload": a.workload, "queries_per_gpu": a.queries,
        "hbm_bytes_per_launch": read_b + write_b,
        "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
        "raw_kb_per_dispatch": {"FETCH_SIZE": {k: v[0] for k, v in fe.items()},
                                "WRITE_SIZE": {k: v[0] for k, v in wr.items()}},
        "dispatches": {"FETCH_SIZE": {k: v[1] for k, v in fe.items()},
                       "WRITE_SIZE": {k: v[1] for k, v in wr.items()}},
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes with --kernel-trace --stats; "
                  "FETCH_SIZE doubled (gfx950 half-count), KB -> bytes; summed over the solve kernels of one run",
    }
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
