# host path after the grouping rewrite: the parity suite's plan-heavy tests, then e2e at
# 125k and 1M with MR_TIMING phases, and the c5 plan create
set -o pipefail
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_scale.py::test_c4_full_scale tests/test_gpu_e2e.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1 && echo tests-ok || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for Q in 125000 1000000; do
MR_TIMING=1 timeout -k 10 300 python bench.py --queries $Q --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 5 > $O/bench_$Q.json 2> $O/bench_$Q.err && echo ok$Q
grep MR_TIMING $O/bench_$Q.err | tail -4
python3 -c "import json;print(json.load(open('$O/bench_$Q.json'))['end_to_end'])"
done
MR_TIMING=1 timeout -k 10 400 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 3 > $O/bench_c5.json 2> $O/bench_c5.err && echo okc5
grep MR_TIMING $O/bench_c5.err | tail -4
python3 -c "import json;d=json.load(open('$O/bench_c5.json'));print(d['value'],d['end_to_end'])"
