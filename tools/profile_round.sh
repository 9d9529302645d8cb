# Profiling recipe of a round: per workload, the bench line, a rocprofv3 kernel
# trace + stats of the same command, and the two PMC passes (FETCH_SIZE, WRITE_SIZE;
# they do not fit one pass on gfx950) summarised into profiles/pmc_<w>.json.
# usage: bash tools/profile_round.sh <round tag, e.g. r02> "<workloads>"
# Outputs under gpurun_out/prof_<tag>/ (copied into profiles/<tag>/ afterwards).
set -o pipefail
TAG=${1:-r02}; WLS=${2:-c4}
O=gpurun_out/prof_$TAG
mkdir -p $O
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
steps() { case $1 in c5) echo 3;; *) echo 20;; esac; }
qpg() { case $1 in c2) echo 10000;; c3) echo 1024;; c4) echo 1000000;; c5) echo 10000;; esac; }
for W in $WLS; do
  ST=$(steps $W)
  timeout -k 10 300 python3 "$R/bench.py" --workload $W --steps $ST --warmup 2 > $O/bench_$W.json 2> $O/bench_$W.err || exit 1
  echo "$W bench ok"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$W -o run --output-format csv -- python3 "$R/bench.py" --workload $W --steps $ST --warmup 2 --no-cpu-baseline > $O/kt_$W.log 2>&1 || exit 1
  echo "$W kernel trace ok"
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --stats -d $O/pmc_${C}_$W -o run --output-format csv -- python3 "$R/bench.py" --workload $W --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_${C}_$W.log 2>&1 || exit 1
  done
  K=""; [ $W = c3 ] && K="--kernels hub_fill_kernel"  # c3 prices the fill (bench.py roofline.kernel)
  python3 "$R/tools/pmc_summary.py" $K --workload $W --queries $(qpg $W) --fetch $O/pmc_FETCH_SIZE_$W --write $O/pmc_WRITE_SIZE_$W --out $O/pmc_$W.json > /dev/null || exit 1
  echo "$W pmc ok"
  K2=hub_kernel; [ $W = c4 ] && K2=hub_lane_kernel; [ $W = c2 ] && K2=hub_group_kernel; [ $W = c3 ] && K2=hub_fill_kernel; [ $W = c5 ] && K2=hub_wide_kernel
  bash "$R/tools/gpu_sq.sh" $W $O/sq_$W && python3 "$R/tools/sq_summary.py" --workload $W --kernel $K2 --sq $O/sq_$W --queries $(qpg $W) --out $O/sq_$W.json > /dev/null || exit 1
  echo "$W sq ok"
done
