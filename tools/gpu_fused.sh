# fused hub+fill all-destinations launch: tests, then A/B against the two-stream overlap
set -o pipefail
mkdir -p gpurun_out/fused
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sssp.py > gpurun_out/fused/tests.log 2>&1 || { tail -30 gpurun_out/fused/tests.log; exit 1; }
tail -2 gpurun_out/fused/tests.log
for i in 1 2; do
  for f in 1 0; do
    MR_FILL_FUSED=$f timeout -k 10 200 python bench.py --workload c3 --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/fused/c3_$f.json 2> gpurun_out/fused/c3_$f.err || exit 1
    echo "fused=$f $(python3 -c "import json;d=json.load(open('gpurun_out/fused/c3_$f.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel_ms'],r['frac'])")"
  done
done
