# GPU: the parity suites, then A/B of the in-tree library against variant(s) on c4, c2, c3 (c5 with C5=1)
set -o pipefail
mkdir -p gpurun_out/aball
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_sssp.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/aball/pytest.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/aball/pytest.log; exit 1; }
for W in c4 c2 c3; do
  echo "== $W"; bash tools/ab_bench.sh "--workload $W --steps 20 --warmup 3" "$@" || exit 1
done
if [ -n "$C5" ]; then echo "== c5"; bash tools/ab_bench.sh "--workload c5 --steps 3 --warmup 1" "$@" || exit 1; fi
