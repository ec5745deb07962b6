#!/bin/bash
# Round-4 session: the 4-wide tree for latency-bound renders (one group per
# pipeline) -- BVH parity tests, C2 at 1 / 20 iterations with and without it,
# the verification of a 1-iteration C2 render.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(tail -c 100 gpurun_out/r4_$n.out | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
step btests 500 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu.py -x -q --timeout 300 --timeout-method thread
B="python3 bench.py --warmup 3 --no-cpu --no-compare --no-count"
for r in 1 2; do
  step lat_b1_r$r 120 $B --steps 1
  WR_BVH_WIDE_LAT=0 step nolat_b1_r$r 120 $B --steps 1
done
step lat_b20 200 $B --steps 20
WR_BVH_VERIFY=1 step lat_verify_b1 200 python3 bench.py --warmup 1 --steps 1 --no-cpu --no-compare
grep -o '"verify[a-z_]*": [0-9]*' gpurun_out/r4_lat_verify_b1.out | head -4
