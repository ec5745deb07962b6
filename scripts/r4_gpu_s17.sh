#!/bin/bash
# Round-4 session: 1-iteration C2 with the 4-wide tree for latency-bound
# renders on / off, alternating, three runs each; the counted line's width.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(grep -o '"width": [0-9]*, "nodes_per_ray": [0-9.]*' gpurun_out/r4_$n.out | head -1)"
  [ $rc -eq 0 ] || exit $rc
}
B="python3 bench.py --warmup 3 --no-cpu --no-compare --no-count"
for r in 1 2 3; do
  step lat2_b1_r$r 120 $B --steps 1
  WR_BVH_WIDE_LAT=0 step nolat2_b1_r$r 120 $B --steps 1
  WR_BVH_WIDE=4 step w4_b1_r$r 120 $B --steps 1
done
step lat2_count 200 python3 bench.py --warmup 1 --steps 1 --no-cpu --no-compare
