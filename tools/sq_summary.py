#!/usr/bin/env python3
"""Summarise a rocprofv3 SQ-counter pass (tools/gpu_sq.sh) into profiles/sq_<workload>.json:
per launch of the workload's dominant kernel, the instruction counts the SQ reports
(SQ_INSTS_VALU / SALU / LDS / VMEM_RD / VMEM_WR, summed over the chip) and the waves.
bench.py turns them into the issue side of the roofline.

    python tools/sq_summary.py --workload c4 --kernel hub_kernel --sq gpurun_out/diag/sq --queries 125000 --out profiles/sq_c4.json
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--kernel", required=True, help="kernel family, e.g. hub_kernel, fill_kernel")
    ap.add_argument("--sq", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--queries", type=int, required=True, help="queries per GPU of the profiled run (bench.py checks it)")
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.sq, "**", "*counter_collection.csv"), recursive=True)
    vals = defaultdict(list)
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                if a.kernel in name and not name.startswith("__amd"):
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {a.kernel} rows under {a.sq}")
    per = {k: sum(v) / len(v) for k, v in vals.items()}
    out = {"workload": a.workload, "queries_per_gpu": a.queries, "kernel": a.kernel, "per_launch": per,
           "launches": max(len(v) for v in vals.values()),
           "method": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD "
                     "SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --stats (tools/gpu_sq.sh); mean per "
                     "dispatch of the kernel family"}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
