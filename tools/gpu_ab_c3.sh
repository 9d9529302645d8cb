# c3 A/B against variant prev (three rounds), after the all-destinations tests
set -o pipefail
mkdir -p gpurun_out/abc3
if [ -z "$NOTEST" ]; then
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sssp.py > gpurun_out/abc3/tests.log 2>&1 || { tail -30 gpurun_out/abc3/tests.log; exit 1; }
tail -1 gpurun_out/abc3/tests.log
fi
for i in 1 2 3; do
  bash tools/ab_bench.sh "--workload c3 --steps 40 --warmup 3" prev || exit 1
done
