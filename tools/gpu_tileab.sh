# fill tile-shape A/B: each variant's fill parity tests, then the c3 bench against the in-tree library
# usage: bash tools/gpu_tileab.sh variant1 [variant2 ...]
set -o pipefail
mkdir -p gpurun_out/tileab
export TMPDIR=/tmp
for v in "$@"; do
  MR_LIB_PATH=marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sssp.py -x -q -k "fill_tiles or ragged or c3" --timeout 300 --timeout-method thread > gpurun_out/tileab/pytest_$v.log 2>&1 && echo "$v tests-ok" || { tail -30 gpurun_out/tileab/pytest_$v.log; exit 1; }
done
bash tools/ab_bench.sh "--workload c3 --steps 20 --warmup 3" "$@"
