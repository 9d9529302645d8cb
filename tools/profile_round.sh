#!/bin/bash
# GPU-box profiling recipe for one round: bench lines, kernel-trace stats and the
# two PMC passes (FETCH_SIZE, WRITE_SIZE) for each workload; outputs under
# gpurun_out/<tag>/, summaries copied into profiles/<tag>/ by the caller.
# Usage (on the box): bash tools/profile_round.sh r01 "c2 c3 c4"
set -euo pipefail
TAG=${1:-r01}
WLS=${2:-"c2 c4"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
cd /tmp
for W in $WLS; do
  K=""
  if [ "$W" = c2 ]; then Q=10000; ST=20; elif [ "$W" = c3 ]; then Q=64; ST=10; K="--kernels fill_kernel";
  elif [ "$W" = c5 ]; then Q=10000; ST=3; else Q=125000; ST=5; fi
  timeout -k 10 400 python3 "$R/bench.py" --workload "$W" --steps "$ST" --warmup 2 > "$O/bench_$W.json" 2> "$O/bench_$W.err"
  echo "bench $W done"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/trace_$W" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload "$W" --steps "$ST" --warmup 2 --no-cpu-baseline > "$O/trace_$W.log" 2>&1
  echo "trace $W done"
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d "$O/pmc_fetch_$W" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload "$W" --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_fetch_$W.log" 2>&1
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --stats -d "$O/pmc_write_$W" -o run --output-format csv -- \
    python3 "$R/bench.py" --workload "$W" --steps 5 --warmup 1 --no-cpu-baseline > "$O/pmc_write_$W.log" 2>&1
  python3 "$R/tools/pmc_summary.py" --workload "$W" --queries "$Q" --fetch "$O/pmc_fetch_$W" \
    --write "$O/pmc_write_$W" --out "$O/pmc_$W.json" $K
  echo "pmc $W done"
done
