#!/bin/bash
# round 4: hub_kernel settle ties without list compares: parity, Fleetfoot rates A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_cert.py > gpurun_out/t_hub.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_new.log 2>&1 || exit 1
MR_LIB_PATH=marshrutka_amd/lib/variants/hubties/libmarshrutka_pf.so timeout -k 10 600 python -u tools/ff_rates.py 1025 125000 3 > gpurun_out/ff_rates_old.log 2>&1
