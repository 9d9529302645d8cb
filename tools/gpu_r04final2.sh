#!/bin/bash
# Round 4 closing box after the host-path changes: the whole GPU suite, smoke(), the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 && echo tests-ok || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke-ok || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo default-ok || exit 1
timeout -k 10 200 python bench.py --workload c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err && echo c2-ok || exit 1
