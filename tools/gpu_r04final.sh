#!/bin/bash
# Round 4 final box: the whole GPU suite, smoke(), profiles of c4 and c2 (bench line, kernel
# trace, PMC, SQ) of the final build, the default bench line, and a 125k-query end to end
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > $O/gpu_tests.log 2>&1 && echo tests-ok || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke-ok || { tail -20 $O/smoke.log; exit 1; }
bash tools/profile_round.sh r04f "c4 c2" || exit 1
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err && echo default-ok || exit 1
MR_TIMING=1 timeout -k 10 200 python bench.py --queries 125000 --steps 10 --warmup 2 --no-cpu-baseline --e2e-reps 5 > $O/bench_125k.json 2> $O/bench_125k.err
