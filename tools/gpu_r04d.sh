# c4 (configs[3], 1M) profiles of the round: bench line, kernel trace, PMC, SQ, SQ waits
set -o pipefail
bash tools/profile_round.sh r04 c4 || exit 1
bash tools/gpu_sq_wait.sh c4 gpurun_out/prof_r04/sqw_c4 && echo sqw-ok
