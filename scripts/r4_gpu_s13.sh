#!/bin/bash
# Round-4 session: C4's hard launches -- the per-step log (tie / scan counts
# and times), then ties one per wave at any count, many-leaf ties handed to the
# wave in the per-lane form (WR_TIE_DEFER=1), and the 4-wide search beside
# them; finally the C4 line with the work counts (its roofline and hbm).
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
V=winmad-s-raytracer-v1.0_amd/variants
B="python3 bench.py --warmup 2 --no-cpu --no-compare --no-count --config c4"
WR_TRACE_LOG=1 step c4_log 300 $B --steps 4
for r in 1 2; do
  step c4_def_r$r 300 $B
  WR_TIE_WAVE_MAX=100000 step c4_tw100k_r$r 300 $B
  WR_LIB=$V/tdefer.so step c4_tdefer_r$r 300 $B
  WR_LIB=$V/w4tdefer.so step c4_w4tdefer_r$r 300 $B
done
step c4_full 400 python3 bench.py --config c4 --no-cpu --no-compare
