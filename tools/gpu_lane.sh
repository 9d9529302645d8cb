# Lane-kernel iteration: parity subset (lane kernel on), c4/c2 bench lines, SQ counters of c4.
# usage: bash tools/gpu_lane.sh <outdir>
set -o pipefail
O=${1:-gpurun_out/lane}
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_full_scale.py -k "auto-lds or lane-lds or lane_kernel or c4_full or kat or edge or invalid or sweep or c2_sample or destinations" > "$O/tests.log" 2>&1 || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
timeout -k 10 120 python bench.py --no-cpu-baseline --e2e-reps 0 > "$O/c4.json" 2> "$O/c4.err" || exit 1
timeout -k 10 120 python bench.py --workload c2 --no-cpu-baseline --e2e-reps 0 > "$O/c2.json" 2> "$O/c2.err" || exit 1
python -c "
import json
for w in ('c4','c2'):
    d=json.load(open('$O/'+w+'.json')); print(w, round(d['value']/1e6,1), 'M q/s', round(d['ms_per_step'],4), 'ms/step', d['roofline']['kernel_ms'])"
bash tools/gpu_sq.sh c4 "$O/sq" && bash tools/gpu_sq_wait.sh c4 "$O/sqw"
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/kt_c2" -o c2 -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload c2 --no-cpu-baseline --e2e-reps 0 --steps 5 > "$GRAFT_REPO_ROOT/$O/kt_c2.log" 2>&1 || exit 1
