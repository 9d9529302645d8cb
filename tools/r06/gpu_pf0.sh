#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r06
for v in base pf0 base pf0; do
  if [ $v = base ]; then L=""; else L="marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so"; fi
  MR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload c4 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/pf_ab_$v.log 2>&1 || { tail -20 gpurun_out/r06/pf_ab_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06/pf_ab_$v.log').read().strip().splitlines()[-1]); print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
  MR_LIB_PATH=$L timeout -k 10 200 python -u bench.py --workload c4 --queries 125000 --steps 50 --warmup 5 --no-cpu-baseline --e2e-reps 0 > gpurun_out/r06/pf_ab_125k_$v.log 2>&1 || { tail -20 gpurun_out/r06/pf_ab_125k_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06/pf_ab_125k_$v.log').read().strip().splitlines()[-1]); print('$v 125k', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
