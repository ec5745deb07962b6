#!/bin/bash
# Round-4 session: k_fast_resolve held to 5 waves per SIMD (96 VGPRs,
# variants/r5.so) against the compiler's 101: C2 at 20 iterations and C4.
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
V=winmad-s-raytracer-v1.0_amd/variants/r5.so
B="python3 bench.py --warmup 2 --no-cpu --no-compare --no-count"
for r in 1 2; do
  step r4_b20_r$r 200 $B --steps 20
  WR_LIB=$V step r5_b20_r$r 200 $B --steps 20
  step r4_c4_r$r 300 $B --config c4
  WR_LIB=$V step r5_c4_r$r 300 $B --config c4
done
