# e2e phases at 125k and 1M, and the certificate's state per slot (Time-first Fleetfoot)
set -o pipefail
O=gpurun_out/r04k
mkdir -p $O
for Q in 125000 1000000; do
MR_TIMING=1 timeout -k 10 300 python bench.py --queries $Q --steps 5 --warmup 1 --no-cpu-baseline --e2e-reps 5 > $O/bench_$Q.json 2> $O/bench_$Q.err && echo ok$Q
grep "MR_TIMING build_plan\|MR_TIMING plan_create" $O/bench_$Q.err | tail -4
python3 -c "import json;print(json.load(open('$O/bench_$Q.json'))['end_to_end'])"
done
for F in 1 2 3; do timeout -k 10 120 python tools/probes/cert_dbg.py $F 2>&1 | grep -v "^$" | tail -20; done
MR_CERT_NOSWEEP=1 timeout -k 10 120 python tools/probes/cert_dbg.py 3 2>&1 | tail -12
