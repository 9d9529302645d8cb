# Round 4, first box: the whole GPU suite on the changed tree (deterministic certificate
# slots, the 1M configs[3] test, the c2 full batch), then the default bench (configs[3],
# 1M queries on one GPU) and its kernel trace.
set -o pipefail
O=gpurun_out/r04a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 && echo tests-ok || { tail -60 $O/gpu_tests.log; }
tail -3 $O/gpu_tests.log
timeout -k 10 400 python bench.py > $O/bench_c4.json 2> $O/bench_c4.err && echo bench-ok || { tail -20 $O/bench_c4.err; exit 1; }
cat $O/bench_c4.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_c4 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 0 > $O/kt_c4.log 2>&1 && echo kt-ok
