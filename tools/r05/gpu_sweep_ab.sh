#!/bin/bash
# timing A/B of sweep variants (Time-first Fleetfoot 1 and 2 at 1025^2 / 125k)
set -o pipefail
mkdir -p gpurun_out
for v in main bs64 bs256 noreq; do
  L=""; [ $v != main ] && L=marshrutka_amd/lib/variants/$v/libmarshrutka_pf.so
  for FF in 1 2; do
    echo -n "$v: "; MR_LIB_PATH=$L timeout -k 10 200 python tools/r05/ff_one.py $FF 1 2 6 || exit 1
  done
done
