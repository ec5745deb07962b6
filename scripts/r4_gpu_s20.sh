#!/bin/bash
# Round-4 session: the 4-wide search held to 5 waves per SIMD (95 VGPRs)
# against 4 (98 VGPRs, variants/f4w4.so): C4 and C2 at 1 iteration (which
# searches the 4-wide tree), alternating; then the BVH parity tests.
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
V=winmad-s-raytracer-v1.0_amd/variants/f4w4.so
B="python3 bench.py --warmup 2 --no-cpu --no-compare --no-count"
for r in 1 2; do
  step f5_c4_r$r 300 $B --config c4
  WR_LIB=$V step f4_c4_r$r 300 $B --config c4
  step f5_b1_r$r 120 $B --steps 1
  WR_LIB=$V step f4_b1_r$r 120 $B --steps 1
done
step f5_tests 400 python -u -m pytest tests/test_gpu_bvh.py -x -q --timeout 300 --timeout-method thread
