#!/bin/bash
# Round-4 session: the -m gpu suite, BVH verification on the bench workloads,
# the piece_min sweep at 1 iteration (overlapped schedule), and the other
# configurations' bench lines.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/r4_$n.out 2> gpurun_out/r4_$n.err
  local rc=$?
  echo "$n rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/r4_$n.out | head -1) $(tail -c 160 gpurun_out/r4_$n.out | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
}
if [ "${SUITE:-1}" = 1 ]; then
  step suite 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
if [ "${VERIFY:-1}" = 1 ]; then
  step verify 400 python3 scripts/verify_bvh.py --out gpurun_out/bvh_verify_r4.json
fi
B="python3 bench.py --warmup 3 --no-cpu --no-compare"
for pm in ${PIECE_MINS:-}; do
  WR_PIECE_MIN=$pm step pm_$pm 120 $B --no-count --steps 1
done
for c in ${CONFIGS:-}; do
  step cfg_$c 300 $B --config $c
done
