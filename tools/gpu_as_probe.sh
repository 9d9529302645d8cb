# all-sources plan size probe: one plan of P sources, with and without the fill's
# bound on concurrently written sources (MR_DBG_FLAGS=32 lifts it)
set -o pipefail
mkdir -p gpurun_out/asp
for P in ${PS:-2048 4096 16384}; do
  for F in ${FLAGS:-0 32}; do
    MR_DBG_FLAGS=$F timeout -k 10 300 python3 tools/all_sources.py --max-plans 1 --per-plan $P --check 4 --oracle 0 > gpurun_out/asp/as_${P}_$F.log 2>&1 || { tail -5 gpurun_out/asp/as_${P}_$F.log; exit 1; }
    echo "P=$P flags=$F $(grep '^plan' gpurun_out/asp/as_${P}_$F.log)"
  done
done
