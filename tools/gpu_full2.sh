# Full GPU suite, then the default bench line
set -o pipefail
O=gpurun_out/full2
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 && echo tests-ok || { tail -30 $O/pytest.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo bench-ok
MR_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_timing.json 2> $O/bench_timing.err && echo timing-ok
MR_HOST_DECODE=1 MR_TIMING=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_timing_host.json 2> $O/bench_timing_host.err && echo timing-host-ok
