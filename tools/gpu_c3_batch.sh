# c3 sources-per-pass sweep: the all-destinations pass at 64..1024 sources (the
# specials' solve of a source is ~85 us of latency whatever the batch; the fill's
# work grows with it).  Outputs under gpurun_out/c3batch/.
set -o pipefail
O=gpurun_out/c3batch
mkdir -p $O
for Q in ${QS:-64 128 256 512 1024}; do
  timeout -k 10 300 python3 bench.py --workload c3 --queries $Q --steps 10 --warmup 2 --no-cpu-baseline \
    > $O/c3_q$Q.json 2> $O/c3_q$Q.err || { tail -20 $O/c3_q$Q.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/c3_q$Q.json')); r=d['roofline']; print($Q, '%.1f G cells/s' % (d['value']/1e9), 'pass %.4f ms' % d['ms_per_step'], 'fill %.4f ms' % r['kernel_ms'], 'frac %.3f' % r['frac'])"
done
