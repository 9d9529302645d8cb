#!/bin/bash
# the final tree: fetch tests, the driver's default bench line, smoke; then the lane
# kernel's pair-table prefetch A/B (variant build, MR_LIB_PATH)
set -o pipefail
mkdir -p gpurun_out/r06
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sssp.py -k "fetch or wire or every_cell" -x -q --timeout 300 --timeout-method thread > gpurun_out/r06/final_tests.log 2>&1 || { tail -30 gpurun_out/r06/final_tests.log; exit 1; }
tail -1 gpurun_out/r06/final_tests.log
timeout -k 10 300 python bench.py > gpurun_out/r06/bench_c4_final2.json 2> gpurun_out/r06/bench_c4_final2.err || { tail -20 gpurun_out/r06/bench_c4_final2.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r06/bench_c4_final2.json'))
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['issue']['valu_busy_frac_at_2_4GHz'], d['parity'])
for k in ('end_to_end','end_to_end_pinned'): print(k, {x: round(d[k][x],3) for x in ('e2e_queries_per_s','ms','plan_create_ms','run_ms','fetch_ms')})"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke2.log 2>&1 || { tail -20 gpurun_out/r06/smoke2.log; exit 1; }
tail -1 gpurun_out/r06/smoke2.log
for v in base pf0 base pf0; do
  if [ $v = base ]; then L=""; else L="marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so"; fi
  MR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/pf_ab_$v.log 2>&1 || { tail -20 gpurun_out/r06/pf_ab_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06/pf_ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
