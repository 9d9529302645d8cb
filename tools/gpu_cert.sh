# Certified fallback on the GPU: its tests, the parity suite's hand-over and Fleetfoot
# cases, the Time-first Fleetfoot rates (tools/ff_rates.py), a kernel trace of ff2
set -o pipefail
O=gpurun_out/cert
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cert.py -x -v --timeout 300 --timeout-method thread > $O/cert.log 2>&1 && echo cert-ok || { tail -40 $O/cert.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_scale.py -x -q -k "fallback or fbsssp or leetfoot" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 && echo parity-ok || { tail -40 $O/parity.log; exit 1; }
timeout -k 10 600 python -u tools/ff_rates.py 1025 125000 3 > $O/ff_rates.log 2>&1 && echo ff-ok || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/cert_prof.py ${FF:-2} 5 > $O/prof.log 2>&1 && echo prof-ok
