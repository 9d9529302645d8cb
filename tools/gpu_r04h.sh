# where the non-linear hub's time goes: Time-first Fleetfoot 3 with the settled specials'
# certification off (MR_DBG_FLAGS=4, an experiment flag) and on, and Legs-first
set -o pipefail
for F in 0 4; do
  MR_DBG_FLAGS=$F timeout -k 10 120 python tools/probes/ff_one.py 3 1 0 || exit 1
  MR_DBG_FLAGS=$F timeout -k 10 120 python tools/probes/ff_one.py 3 0 2 || exit 1
done
MR_HUB_SPW=1 timeout -k 10 120 python tools/probes/ff_one.py 3 1 0
