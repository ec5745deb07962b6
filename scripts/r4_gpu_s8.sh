#!/bin/bash
# Round-4 session: k_fast_hard's tie / scan grid for latency-bound steps --
# WR_TIE_WAVE_MAX (ties one per wave up to this many) x WR_SCAN_WAVES, at 1
# and 20 iterations.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1)"
  [ $rc -eq 0 ] || exit $rc
}
B="python3 bench.py --warmup 3 --no-cpu --no-compare --no-count"
for r in 1 2; do
  for tw in "512 256" "4096 256" "4096 1024" "100000 1024" "100000 4096"; do
    set -- $tw
    WR_TIE_WAVE_MAX=$1 WR_SCAN_WAVES=$2 step tw$1_s$2_b1_r$r 120 $B --steps 1
  done
done
for tw in "512 256" "4096 1024" "100000 1024"; do
  set -- $tw
  WR_TIE_WAVE_MAX=$1 WR_SCAN_WAVES=$2 step tw$1_s$2_b20 200 $B --steps 20
done
