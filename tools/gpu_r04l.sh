# lane kernel without per-cell records (rank by formula, specials by scan): lane parity
# modes, the 1M configs[3] test, A/B against MR_RANK_TABLE=1 and the c4 PMC traffic;
# then the N>1 bench path: gloo with two ranks on the one GPU, RCCL at world size 1
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "lane" tests/test_gpu_full_scale.py -k "lane or c4_full" -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 && echo tests-ok || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in std tab std tab; do
  E=""; [ $v = tab ] && E="MR_RANK_TABLE=1"
  env $E timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --e2e-reps 0 > $O/ab_$v.json 2> $O/ab_$v.err || exit 1
  echo "$v $(python3 -c "import json;d=json.load(open('$O/ab_$v.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'])")"
done
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-trace --stats -d $O/pmc_$C -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > $O/pmc_$C.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py --workload c4 --queries 1000000 --fetch $O/pmc_FETCH_SIZE --write $O/pmc_WRITE_SIZE --out $O/pmc_c4.json > /dev/null && echo pmc-ok
python3 -c "import json;d=json.load(open('$O/pmc_c4.json'));print('pmc', d['hbm_bytes_per_launch'], d['read_bytes_per_launch'], d['write_bytes_per_launch'])"
for W in c2 c4; do
  MR_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --workload $W > $O/bench_n2_$W.json 2> $O/bench_n2_$W.err && echo n2-$W-ok || { tail -20 $O/bench_n2_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_n2_$W.json'));print('$W',d['value'],d['ms_per_step'],d['scaling'],d['config']['queries_per_gpu'],d.get('gather_check'))"
  MR_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --workload $W --steps 10 --warmup 2 --no-cpu-baseline > $O/rccl1_$W.json 2> $O/rccl1_$W.err || { tail -20 $O/rccl1_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/rccl1_$W.json'));print('rccl1 $W',d['value'],d['ms_per_step'],d.get('gather_check'))"
done
