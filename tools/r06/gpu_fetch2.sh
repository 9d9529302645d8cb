#!/bin/bash
# fresh-plan fetch with fewer host threads; region-table kernel trace
set -o pipefail
mkdir -p gpurun_out/r06
for t in 8 4; do
  MR_HOST_THREADS=$t FRESH=1 MR_TIMING=1 timeout -k 10 300 python -u tools/r06/fetch_time.py > gpurun_out/r06/fetch_fresh_t$t.log 2>&1 || { tail -20 gpurun_out/r06/fetch_fresh_t$t.log; exit 1; }
  echo "threads $t"; grep "MR_FETCH_WIRE" gpurun_out/r06/fetch_fresh_t$t.log
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06/prof_region -o run --output-format csv -- python3 tools/r06/region_time.py c4 c5 > gpurun_out/r06/prof_region.log 2>&1 || { tail -20 gpurun_out/r06/prof_region.log; exit 1; }
f=$(find gpurun_out/r06/prof_region -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r06/region_kernel_stats.csv
python3 - <<'P'
import csv
for r in csv.DictReader(open("gpurun_out/r06/region_kernel_stats.csv")):
    print(r["Name"][:50], r["Calls"], r["TotalDurationNs"], r["AverageNs"])
P
