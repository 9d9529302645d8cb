set -o pipefail
mkdir -p gpurun_out/align
for r in 1 2; do
for A in 32 64; do
  MR_REC_ALIGN=$A timeout -k 10 300 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/align/c3_$A.json 2> gpurun_out/align/c3_$A.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/align/c3_$A.json'));r=d['roofline'];print('align $A', d['value']/1e9, d['ms_per_step'], r['kernel_ms'], r['frac'])"
done
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_sssp.py -x -q --timeout 300 --timeout-method thread > gpurun_out/align/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/align/pytest.log; exit $rc
