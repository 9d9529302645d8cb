# a quick correctness gate (parity tests that read the written counter), then
# c4 / c2 / c3 A/B against variants.  usage: bash tools/gpu_ab3.sh variant1 [...]
set -o pipefail
mkdir -p gpurun_out/ab3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sssp.py -x -q -k "not every_cell and not fill_tiles" --timeout 300 --timeout-method thread > gpurun_out/ab3/pytest.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/ab3/pytest.log; exit 1; }
for w in "c4 --steps 10 --warmup 2" "c2 --steps 50 --warmup 5" "c3 --steps 20 --warmup 3"; do
  echo "== $w"; bash tools/ab_bench.sh "--workload $w" "$@" || exit 1
done
