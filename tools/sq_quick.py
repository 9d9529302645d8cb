"""Per-kernel averages of a rocprofv3 counter-collection CSV (quick look while iterating).
usage: python tools/sq_quick.py <dir> [kernel substring]"""
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "lane"
for f in glob.glob(d + "/**/*counter_collection*.csv", recursive=True):
    acc, ids = {}, {}
    for r in csv.DictReader(open(f)):
        if sub not in r.get("Kernel_Name", ""):
            continue
        c = r["Counter_Name"]
        acc[c] = acc.get(c, 0.0) + float(r["Counter_Value"])
        ids.setdefault(c, set()).add(r.get("Dispatch_Id"))
    for c in sorted(acc):
        print(f"{c:24s} {acc[c] / len(ids[c]):16.0f}  ({len(ids[c])} dispatches)")
