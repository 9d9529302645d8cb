# e2e phase timings at 1M and 125k (MR_TIMING=1), and the select-chain micro-benchmark
set -o pipefail
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 120 ./tools/micro/select_chain > $O/select_chain.txt 2>&1; echo "micro rc=$?"
cat $O/select_chain.txt
MR_TIMING=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 3 > $O/bench_1m.json 2> $O/bench_1m.err && echo ok1
grep MR_TIMING $O/bench_1m.err | tail -12
MR_TIMING=1 timeout -k 10 300 python bench.py --queries 125000 --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 3 > $O/bench_125k.json 2> $O/bench_125k.err && echo ok2
grep MR_TIMING $O/bench_125k.err | tail -12
python -c "import json;[print(f, json.load(open('$O/'+f))['end_to_end']) for f in ('bench_1m.json','bench_125k.json')]"
