#!/bin/bash
# round 4: wide kernel settle ties without list compares: parity (wide modes, c5 full scale), c5 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py -k "wide or many_campfires" > gpurun_out/t_wide.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_full_scale.py -k "c5" >> gpurun_out/t_wide.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/b_c5_new.json 2> gpurun_out/b_c5_new.err || exit 1
MR_LIB_PATH=marshrutka_amd/lib/variants/wideties/libmarshrutka_pf.so timeout -k 10 300 python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline --e2e-reps 0 > gpurun_out/b_c5_old.json 2> gpurun_out/b_c5_old.err
