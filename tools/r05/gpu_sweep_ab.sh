#!/bin/bash
# A/B of the sweep variants on the flagged Fleetfoot 1 / 2 sources
set -o pipefail
mkdir -p gpurun_out
run() {  # tag lib flags
  echo "$1 flags=$3"
  MR_LIB_PATH=$2 MR_DBG_FLAGS=$3 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_cert.py -k "flagged_source_certified_1025" > gpurun_out/ab_$1_$3.log 2>&1; tail -n 1 gpurun_out/ab_$1_$3.log
}
run main "" 0
run main "" 512
run main "" 3072
run helper marshrutka_amd/lib/variants/helper/libmarshrutka_pf.so 0
