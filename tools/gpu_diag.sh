# c4 diagnostics: per-phase cycle stamps of the hub kernel (diag build) and SQ counters
set -o pipefail
O=gpurun_out/diag; mkdir -p $O
MR_LIB_PATH=marshrutka_amd/lib/diag/libmarshrutka_pf.so timeout -k 10 300 python bench.py --workload ${W:-c4} --steps 3 --warmup 1 --no-cpu-baseline > $O/stamps.json 2> $O/stamps.err && echo stamps-ok
bash tools/gpu_sq.sh ${W:-c4} $O/sq && echo sq-ok
