#!/bin/bash
# kernel traces of the certified fallback at Fleetfoot 2 and 1, Time first (queued sweep; full sweep A/B)
set -o pipefail
mkdir -p gpurun_out/certprof
export TMPDIR=/tmp
for FF in 2 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/certprof/ff$FF -o run --output-format csv -- python3 tools/r05/ff_one.py $FF 1 2 5 > gpurun_out/certprof/ff$FF.log 2>&1 || exit 1
  grep "pass" gpurun_out/certprof/ff$FF.log
done
MR_DBG_FLAGS=256 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/certprof/ff2full -o run --output-format csv -- python3 tools/r05/ff_one.py 2 1 2 5 > gpurun_out/certprof/ff2full.log 2>&1 || exit 1
grep "pass" gpurun_out/certprof/ff2full.log
for d in ff2 ff1 ff2full; do echo $d; head -12 gpurun_out/certprof/$d/run_kernel_stats.csv | cut -d, -f1-6; done
