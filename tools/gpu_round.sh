# parity tests, then the profiling recipe for the given workloads
set -o pipefail
mkdir -p gpurun_out/rt
timeout -k 10 900 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -q --timeout 300 --timeout-method thread > gpurun_out/rt/pytest.log 2>&1 && echo tests-ok || { tail -30 gpurun_out/rt/pytest.log; exit 1; }
bash tools/profile_round.sh r01 "$1"
