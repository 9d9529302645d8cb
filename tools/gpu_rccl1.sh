# The N > 1 bench path on RCCL at world size 1 (MR_BENCH_DIST=1): process group,
# double-buffered gather, gather check — on the one GPU of the box
set -o pipefail
mkdir -p gpurun_out/rccl1
for W in c2 c4; do
  MR_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --workload $W --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/rccl1/$W.json 2> gpurun_out/rccl1/$W.err || { tail -20 gpurun_out/rccl1/$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/rccl1/$W.json'));print('$W',d['value'],d['ms_per_step'],d['config'].get('gather_check'))"
done
