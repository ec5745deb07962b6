#!/bin/bash
# Round-4 session: C4's hard-launch knobs on the final build -- ties one per
# wave up to 1,024 / 4,096 / 16,384, scan waves 256 / 1,024.
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
B="python3 bench.py --warmup 2 --no-cpu --no-compare --no-count --config c4"
for r in 1 2; do
  step k_def_r$r 300 $B
  WR_TIE_WAVE_MAX=1024 step k_tw1k_r$r 300 $B
  WR_TIE_WAVE_MAX=16384 step k_tw16k_r$r 300 $B
  WR_SCAN_WAVES=1024 step k_sw1k_r$r 300 $B
done
