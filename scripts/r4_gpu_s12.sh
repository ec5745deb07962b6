#!/bin/bash
# Round-4 session: the 4-wide search tree with a short LDS stack (+ global
# spill) against the binary default -- C2 at 20 iterations with the work
# counts, C4 at 64.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(grep -o '"nodes_per_ray": [0-9.]*, "tests_per_ray": [0-9.]*' gpurun_out/r4_$n.out | head -1)"
  [ $rc -eq 0 ] || exit $rc
}
B="python3 bench.py --warmup 3 --no-cpu --no-compare"
V=winmad-s-raytracer-v1.0_amd/variants
for r in 1 2; do
  step w2_b20_r$r 200 $B --steps 20
  for v in w4s12 w4s16 w4s24; do
    WR_LIB=$V/$v.so step ${v}_b20_r$r 200 $B --steps 20
  done
done
step w2_c4 300 $B --config c4 --no-count
for v in w4s12 w4s16; do
  WR_LIB=$V/$v.so step ${v}_c4 300 $B --config c4 --no-count
done
