#!/bin/bash
# round 5: LDS bank conflicts and wait states of the c4 lane kernel (one --pmc pass of 8 SQ counters)
set -o pipefail
mkdir -p gpurun_out/sq_lds
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/sq_lds -o run --output-format csv -- python3 "$R/bench.py" --workload c4 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/sq_lds/log.txt 2>&1 || { tail -20 gpurun_out/sq_lds/log.txt; exit 1; }
python3 "$R/tools/sq_quick.py" gpurun_out/sq_lds lane
