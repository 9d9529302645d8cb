# SQ instruction counters for one workload's kernels (one --pmc pass)
# usage: bash tools/gpu_sq.sh <workload> <outdir>
set -o pipefail
W=${1:-c3}; O=${2:-gpurun_out/sq_$W}
mkdir -p "$O"
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --stats -d "$O" -o run --output-format csv -- python3 "$R/bench.py" --workload "$W" --steps 3 --warmup 1 --no-cpu-baseline > "$O/log.txt" 2>&1
