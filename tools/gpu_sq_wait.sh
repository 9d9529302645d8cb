# Where the hub kernel's waves spend their cycles (one --pmc pass, 8 SQ counters):
# parked on s_waitcnt/barriers, stalled at issue, or issuing (by unit)
# usage: bash tools/gpu_sq_wait.sh <workload> <outdir>
set -o pipefail
W=${1:-c4}; O=${2:-gpurun_out/sqw_$W}
mkdir -p "$O"
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --kernel-trace --stats -d "$O" -o run --output-format csv -- python3 "$R/bench.py" --workload "$W" --steps 3 --warmup 1 --no-cpu-baseline > "$O/log.txt" 2>&1
