# query-mode change: hub parity tests, then A/B c2 and c4 against variant prev (twice each)
set -o pipefail
mkdir -p gpurun_out/abq
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/abq/tests.log 2>&1 || { tail -30 gpurun_out/abq/tests.log; exit 1; }
tail -2 gpurun_out/abq/tests.log
for W in ${WL:-c2 c4}; do
  for i in 1 2; do
    bash tools/ab_bench.sh "--workload $W --steps 20 --warmup 3" prev || exit 1
  done
done
